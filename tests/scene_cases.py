"""TEST INFRASTRUCTURE: generic scenes (oracle bodies) shared by the CPU
emulation tests and the GPU parity tests."""
import numpy as np


def straddle_scene(theta):
    """A falling dynamic quad (body 0, vertex items 0..3) over a static,
    rotated body 1 of 14 far-away quads and a hexagonal floor under the quad
    (vertex items 60..65): at one env per wave the floor straddles phase T's
    first two 64-item chunks.  theta rotates body 1: its world
    vertex order is a re-sort of the local order."""
    from cotix_oracle import geometry as G
    from cotix_oracle import physics as P
    c, s = np.cos(-theta), np.sin(-theta)

    def local(pts):  # world points of body 1 (at the origin) -> its local frame
        return [(float(np.float32(x * c - y * s)), float(np.float32(x * s + y * c))) for x, y in pts]

    dummies = [G.Polygon(local([(40 + 5 * i, 0), (42 + 5 * i, 0), (42 + 5 * i, 2), (40 + 5 * i, 2)]), kind="Polygon4")
               for i in range(14)]
    floor = G.Polygon(local([(-3, -1), (3, -1), (3.2, -0.5), (3, 0), (-3, 0), (-3.2, -0.5)]), kind="Polygon6")
    box = G.Polygon([(-0.5, 0.0), (0.5, 0.0), (0.5, 0.6), (-0.5, 0.6)], kind="Polygon4")
    return [P.Body([box], mass=1.0, inertia=1.0, position=(0.1, 0.05), velocity=(0.0, -0.5), angular_velocity=0.3,
                   elasticity=0.5, friction_coefficient=0.2),
            P.Body(dummies + [floor], mass=float("inf"), inertia=float("inf"), angle=theta, elasticity=0.5,
                   friction_coefficient=0.2)]


def mixed_scene(circle):
    """Two quads falling onto a static AABB floor (one in contact with the
    other), optionally a ball: AABB x polygon (and circle x polygon) contacts."""
    from cotix_oracle import geometry as G
    from cotix_oracle import physics as P
    quad = [(-0.5, 0.0), (0.5, 0.0), (0.5, 0.6), (-0.5, 0.6)]
    bodies = [P.Body([G.Polygon(quad, kind="Polygon4")], position=(0.1, 0.02), velocity=(0.0, -0.4),
                     angular_velocity=0.2, elasticity=0.5, friction_coefficient=0.2),
              P.Body([G.Polygon(quad, kind="Polygon4")], position=(0.95, 0.3), angle=0.3, velocity=(-0.2, -0.3),
                     elasticity=0.5, friction_coefficient=0.2),
              P.Body([G.AABB((-4.0, -1.0), (4.0, 0.0))], mass=float("inf"), inertia=float("inf"), elasticity=0.5,
                     friction_coefficient=0.2)]
    if circle:
        bodies.insert(2, P.Body([G.Circle(0.3, (0.0, 0.0))], position=(-0.75, 0.25), velocity=(0.3, -0.2),
                                elasticity=0.5, friction_coefficient=0.2))
    return bodies


def octagon_row(n):
    """n octagon bodies in a row, neighbours overlapping (every pair of
    neighbours in contact), body 0 static: a polygon scene whose step tile
    needs more LDS than 4 envs per wave give (n = 9: one env per wave fits,
    n = 12: nothing fits -- rejected at cotix_scene_create)."""
    from cotix_oracle import geometry as G
    from cotix_oracle import physics as P
    a = np.arange(8) * (2 * np.pi / 8)
    octa = [(float(np.float32(0.25 * np.cos(t))), float(np.float32(0.25 * np.sin(t)))) for t in a]
    out = [P.Body([G.Polygon(octa, kind="Polygon")], mass=float("inf"), inertia=float("inf"), elasticity=0.5,
                  friction_coefficient=0.2)]
    for i in range(1, n):
        out.append(P.Body([G.Polygon(octa, kind="Polygon")], position=(0.46 * i, 0.02 * i), angle=0.1 * i,
                          velocity=(0.1 * (i % 3) - 0.1, -0.2), angular_velocity=0.05 * i, elasticity=0.5,
                          friction_coefficient=0.2))
    return out


def polygon20():
    """20 polygon parts over 5 bodies: a static terrain body of 8 quads and
    4 dynamic bodies of a hexagon and 2 quads each, resting on and against
    one another -- a scene whose tiles fit the LDS only in workgroups of
    fewer than 4 waves (cotix_scene_waves_per_group)."""
    from cotix_oracle import geometry as G
    from cotix_oracle import physics as P
    terrain = []
    for k in range(8):
        x0, x1 = -4.0 + k, -3.0 + k
        terrain.append(G.Polygon([(x0, -1.0), (x1, -1.0), (x1, 0.05 * (k % 3)), (x0, 0.05 * ((k + 1) % 3))],
                                 kind="Polygon4"))
    out = [P.Body(terrain, mass=float("inf"), inertia=float("inf"), elasticity=0.3, friction_coefficient=0.4)]
    hexv = [(0.3 * np.cos(t), 0.3 * np.sin(t)) for t in np.arange(6) * (np.pi / 3)]
    for i in range(4):
        parts = [G.Polygon(hexv, kind="Polygon6"),
                 G.Polygon([(0.2, -0.1), (0.5, -0.1), (0.5, 0.1), (0.2, 0.1)], kind="Polygon4"),
                 G.Polygon([(-0.5, -0.1), (-0.2, -0.1), (-0.2, 0.1), (-0.5, 0.1)], kind="Polygon4")]
        out.append(P.Body(parts, mass=1.0 + 0.5 * i, inertia=0.5 + 0.25 * i, position=(-2.6 + 1.3 * i, 0.33),
                          angle=0.2 * i, velocity=(0.1 * (i % 2) - 0.05, -0.3), angular_velocity=0.1 * i,
                          elasticity=0.4, friction_coefficient=0.3))
    return out
