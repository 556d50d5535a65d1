"""Render export: env.draw(painter) without host callbacks.

The reference draws from inside jit through jax.debug.callback into a
pygame PyPainter (cotix/_viz.py:6-75): RoboCupEnv.draw (cotix/_robocup.py:
140-150) fills every body with its colour and outlines it with its edge
colour; LunarLander.draw (cotix/_lunar_lander.py:220-225) draws every body
with the shapes' default colours plus two red lines.  Here the per-env
geometry of those draws is one device kernel (cotix_render: every part
transformed by its body -- circles as (cx, cy, r), AABB and polygon edges in
get_edges order) and the static part -- which primitive, which colour, in
which order -- is a command list built once per scenario.  replay() issues the
reference's exact Painter call sequence for one env from that table, so any
object with draw_circle / draw_line / next (a PyPainter included) works.
"""
import torch

from . import _ffi
from .shapes import AABB, AbstractPolygon, Circle

# default colours of the shapes' draw() (cotix/_convex_shapes.py:43,119,189)
DEFAULT_COLOR = {"circle": (128, 128, 128), "aabb": (128, 128, 128), "polygon": (255, 255, 255)}


def _kind(part):
    if isinstance(part, Circle):
        return "circle"
    if isinstance(part, AABB):
        return "aabb"
    if isinstance(part, AbstractPolygon):
        return "polygon"
    raise TypeError("unknown part type %r" % type(part))


def part_layout(bodies):
    """[(kind, first primitive, primitive count)] per part, parts in scene
    order (the kernel's layout: circle 1, AABB 4, polygon n primitives)."""
    out, off = [], 0
    for b in bodies:
        for p in b.shape.parts:
            k = _kind(p)
            n = 1 if k == "circle" else (4 if k == "aabb" else p.vertices.shape[-2])
            out.append((k, off, n))
            off += n
    return out


def render(world, dyn=None):
    """f32 [B, n_prims, 4] on the world's device: the transformed geometry of
    every drawn primitive of every env (cotix_render)."""
    d = world.dyn if dyn is None else dyn
    n = _ffi.lib.cotix_render_count(world.scene.handle)
    if n < 0:
        _ffi.check(n, "cotix_render_count")
    layout = part_layout(world.bodies)
    if layout and layout[-1][1] + layout[-1][2] != n:
        raise RuntimeError("render layout mismatch with the library")
    out = torch.empty(world.B, n, 4, dtype=torch.float32, device=world.device)
    _ffi.check(_ffi.lib.cotix_render(world.scene.handle, _ffi.ptr(d), _ffi.ptr(world.geom), world.geom_stride,
                                     world.B, _ffi.ptr(out), _ffi.stream_ptr(world.device)), "cotix_render")
    return out


def _shape_cmds(layout, parts_of_body, color):
    """UniversalShape.draw(painter, [color]) -> part.transform(T).draw(...)."""
    cmds = []
    for p in parts_of_body:
        k, off, n = layout[p]
        c = DEFAULT_COLOR[k] if color is None else color
        if k == "circle":
            cmds.append(("circle", off, c))
        else:  # AABB.draw and Polygon.draw both draw their edges
            cmds.extend(("line", off + q, c) for q in range(n))
    return cmds


def _edge_cmds(layout, parts_of_body, color):
    """UniversalShape.drawEdges(painter, color=...)."""
    cmds = []
    for p in parts_of_body:
        k, off, n = layout[p]
        if k == "circle":
            raise NotImplementedError("Circle.drawEdges (cotix/_convex_shapes.py:46-47)")
        cmds.extend(("line", off + q, color) for q in range(n))
    return cmds


def _parts_by_body(bodies):
    out, p = [[] for _ in bodies], 0
    for i, b in enumerate(bodies):
        for _ in b.shape.parts:
            out[i].append(p)
            p += 1
    return out


def commands_bodies(bodies, colors=None, edge_colors=None, extra_lines=()):
    """The draw command list of `for body: shape.draw(color); shape.drawEdges(edge_color)`
    then static lines.  colors / edge_colors: per body, None = default / no edge pass."""
    layout = part_layout(bodies)
    pb = _parts_by_body(bodies)
    cmds = []
    for i in range(len(bodies)):
        cmds.extend(_shape_cmds(layout, pb[i], None if colors is None else colors[i]))
        if edge_colors is not None and edge_colors[i] is not None:
            cmds.extend(_edge_cmds(layout, pb[i], edge_colors[i]))
    for (a, b, c) in extra_lines:
        cmds.append(("static_line", (a, b), c))
    return cmds


def replay(painter, cmds, prims, env=0):
    """Issue the Painter calls of one env; prims: the render() output (any
    device; moved to the host here), then painter.next() as the reference's
    draw() ends with."""
    g = prims[env].detach().to("cpu").tolist() if isinstance(prims, torch.Tensor) else prims[env]
    for op, ref, color in cmds:
        if op == "circle":
            x, y, r, _ = g[ref]
            painter.draw_circle((x, y), r, color)
        elif op == "line":
            x0, y0, x1, y1 = g[ref]
            painter.draw_line((x0, y0), (x1, y1), color)
        else:
            painter.draw_line(ref[0], ref[1], color)
    painter.next()


class RecordingPainter:
    """A Painter that records its calls (tests, headless use)."""

    def __init__(self):
        self.calls = []

    def draw_circle(self, center, radius, color):
        self.calls.append(("circle", tuple(center), radius, tuple(color)))

    def draw_line(self, start, end, color):
        self.calls.append(("line", tuple(start), tuple(end), tuple(color)))

    def draw_polygon(self, vertices, color):
        self.calls.append(("polygon", [tuple(v) for v in vertices], tuple(color)))

    def next(self):
        self.calls.append(("next",))
