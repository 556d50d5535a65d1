"""TEST INFRASTRUCTURE ONLY -- restatement of the reference's env.draw(painter)
call sequence (the checker of parallax_amd.render; never shipped).

  RoboCupEnv.draw      cotix/_robocup.py:131-150
  LunarLander.draw     cotix/_lunar_lander.py:220-225
  AbstractBody.draw    cotix/_bodies.py:131-132
  UniversalShape.draw / drawEdges   cotix/_universal_shape.py:79-85
  Circle.draw :43-44, AABB.draw/drawEdges :119-133, Polygon.draw/drawEdges :189-194
  get_edges: AABB :82-93, Polygon :160-163
"""
from . import geometry as G

ROBOCUP_COLORS = [(0, 180, 0)] * 2 + [(255, 255, 0), (0, 128, 255), (255, 0, 0)]
ROBOCUP_EDGE_COLORS = [(255, 255, 255)] * 2 + [(255, 255, 0), (0, 128, 255), None]


def _draw_shape(calls, shape, color=None):
    if isinstance(shape, G.Circle):
        calls.append(("circle", tuple(shape.position), shape.radius, color or (128, 128, 128)))
    else:  # AABB.draw -> drawEdges (default grey); Polygon.draw -> drawEdges (default white)
        c = color or ((128, 128, 128) if isinstance(shape, G.AABB) else (255, 255, 255))
        for e0, e1 in shape.edges():
            calls.append(("line", tuple(e0), tuple(e1), c))


def _draw_edges(calls, shape, color):
    if isinstance(shape, G.Circle):
        raise NotImplementedError
    for e0, e1 in shape.edges():
        calls.append(("line", tuple(e0), tuple(e1), color))


def robocup_draw(bodies):
    calls = []
    for ec, c, b in zip(ROBOCUP_EDGE_COLORS, ROBOCUP_COLORS, bodies):
        T = b.transformer()
        for p in b.parts:
            _draw_shape(calls, p.transform(T), c)
        if ec is not None:
            for p in b.parts:
                _draw_edges(calls, p.transform(T), ec)
    calls.append(("next",))
    return calls


def lunar_lander_draw(bodies):
    calls = []
    for b in bodies:
        T = b.transformer()
        for p in b.parts:
            _draw_shape(calls, p.transform(T))
    calls.append(("line", (-2, -1.8), (-2, -1.0), (255, 0, 0)))
    calls.append(("line", (2, -1.8), (2, -1.0), (255, 0, 0)))
    calls.append(("next",))
    return calls
