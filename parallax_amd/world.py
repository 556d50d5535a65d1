"""A batched world: one compiled scene + SoA device state for B envs.

Layout in HBM (DESIGN.md "Data layout"):
  dyn   f32 [n_bodies][6][B]   px, py, vx, vy, angle, angular_velocity
  keys  i32 [B][2]             collider PRNG key per env (uint32 bits)
  err   i32 [B]                error bits (cotix/_contacts.py:105-107 trips)
  geom  f32 [G] shared or [B][G] per env: local part geometry
"""
import torch

from . import _ffi
from .bodies import AnyBody, BodyView
from .params import DEFAULT as DEFAULT_PARAMS
from .params import CotixParams, Params
from .shapes import AbstractPolygon


# the step kernel's scene specializations (cxk::SPEC_*, cotix_kernel.h)
SPECIALIZATIONS = ("generic", "robocup", "lunar", "robocup_partitionable", "lunar_partitionable", "box")


class Scene:
    """cotix_scene_create_ex: the collider's trace-time enumeration
    (cotix/_colliders.py:86-131) compiled once into device tables, with the
    parameter block `params` (parallax_amd.Params; None: the reference's
    literals)."""

    def __init__(self, bodies, params=None):
        import ctypes
        self.params = DEFAULT_PARAMS if params is None else params
        if not isinstance(self.params, Params):
            raise TypeError("params must be a parallax_amd.Params")
        self.n_bodies = len(bodies)
        # per-env body parameters (a [B] tensor in some body): carried in each
        # env's geometry row (include/cotix_amd.h COTIX_SCENE_PER_ENV_BODY_PARAMS)
        self.per_env_params = any(b.params_per_env() for b in bodies)
        params = torch.tensor([b.template_params() for b in bodies], dtype=torch.float32)
        part_body, part_type, part_nv = [], [], []
        for i, b in enumerate(bodies):
            for p in b.shape.parts:
                part_body.append(i)
                part_type.append(p.type_id)
                part_nv.append(p.vertices.shape[-2] if isinstance(p, AbstractPolygon) else 0)
        self.parts = [p for b in bodies for p in b.shape.parts]
        pb = torch.tensor(part_body, dtype=torch.int32)
        pt = torch.tensor(part_type, dtype=torch.int32)
        pn = torch.tensor(part_nv, dtype=torch.int32)
        h = ctypes.c_void_p()
        cp = self.params.c_struct()
        flags = _ffi.SCENE_PER_ENV_BODY_PARAMS if self.per_env_params else 0
        _ffi.check(_ffi.lib.cotix_scene_create_ex2(self.n_bodies, _ffi.ptr(params), len(part_body), _ffi.ptr(pb),
                                                   _ffi.ptr(pt), _ffi.ptr(pn), ctypes.byref(cp), flags,
                                                   ctypes.byref(h)), "cotix_scene_create_ex2")
        self.handle = h
        self.geom_floats = _ffi.lib.cotix_scene_geom_floats(h)

    def info(self):
        import ctypes
        v = [ctypes.c_int() for _ in range(4)]
        _ffi.check(_ffi.lib.cotix_scene_info(self.handle, *[ctypes.byref(x) for x in v]), "cotix_scene_info")
        return dict(zip(("contacts", "cells", "candidates", "types"), [x.value for x in v]))

    def compiled_params(self):
        """The scene's parameter block as the library holds it (cotix_scene_params)."""
        import ctypes
        c = CotixParams()
        _ffi.check(_ffi.lib.cotix_scene_params(self.handle, ctypes.byref(c)), "cotix_scene_params")
        return Params.from_c(c)

    def set_variant(self, envs_per_wave=0, specialize=True):
        """Kernel variant of this scene's launches: envs per wave (0 = the
        default 4; 1, 2, 4, 8) and whether the reference scenes may use their
        specialized kernels.  Every variant computes the same bits."""
        _ffi.check(_ffi.lib.cotix_scene_set_variant(self.handle, int(envs_per_wave), 1 if specialize else 0),
                   "cotix_scene_set_variant")

    def variant(self):
        """What a step launch uses: {"envs_per_wave": EW, "specialization":
        one of SPECIALIZATIONS} -- the reference scenes under the default
        constants get a kernel with their whole header folded in, per PRNG
        layout."""
        import ctypes
        ew, sp = ctypes.c_int(), ctypes.c_int()
        _ffi.check(_ffi.lib.cotix_scene_variant(self.handle, ctypes.byref(ew), ctypes.byref(sp)),
                   "cotix_scene_variant")
        return {"envs_per_wave": ew.value, "specialization": SPECIALIZATIONS[sp.value]}

    def waves_per_group(self):
        """Waves per workgroup of this scene's launches: 4 (one per SIMD), or 2
        / 1 when its tiles do not fit the LDS four at a time (large scenes)."""
        return _ffi.lib.cotix_scene_waves_per_group(self.handle)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and _ffi is not None and _ffi.lib is not None:
            _ffi.lib.cotix_scene_destroy(h)
            self.handle = None


class World:
    @classmethod
    def from_bodies(cls, bodies, batch=None, device="cuda", keys=None, params=None):
        """A World from the reference's own body pytrees (a list of AnyBody
        objects, or an env object with ``.bodies``), read by the reference's
        class and field names (parallax_amd.pytree); leaves with a leading
        batch dimension (a vmapped pytree) give the env axis."""
        from .pytree import bodies_from_reference
        pb, B = bodies_from_reference(bodies, batch)
        return cls(pb, B, device, keys, params)

    def __init__(self, bodies, batch=1, device="cuda", keys=None, params=None):
        if not all(isinstance(b, AnyBody) for b in bodies):
            raise TypeError("bodies must be AnyBody")
        self.bodies = list(bodies)
        self.B = int(batch)
        self.device = torch.device(device)
        self.scene = Scene(self.bodies, params)
        self.params = self.scene.params
        self.geom = self._upload_geometry()
        self.geom_stride = 0 if self.geom.dim() == 1 else self.geom.shape[1]
        self.dyn = torch.stack([b.dyn_columns(self.B) for b in self.bodies], 0).to(self.device).contiguous()
        if keys is not None and tuple(keys.shape) != (self.B, 2):
            raise ValueError("keys must be [B, 2] = [%d, 2], got %s" % (self.B, tuple(keys.shape)))
        self.keys = (keys if keys is not None else torch.zeros(self.B, 2, dtype=torch.int32)).to(
            self.device, torch.int32).contiguous()
        self.err = torch.zeros(self.B, dtype=torch.int32, device=self.device)

    # -- geometry ---------------------------------------------------------
    def _upload_geometry(self):
        cols, batched = [], False
        for p in self.scene.parts:
            g = p.local_geometry()
            batched = batched or g.dim() == 2
            cols.append(g)
        if self.scene.per_env_params:  # each env's [n_bodies][4] parameters after its parts' words
            batched = True
            cols.append(torch.cat([b.param_columns(self.B).T for b in self.bodies], dim=1))
        if batched:
            cols = [c.expand(self.B, -1) if c.dim() == 1 else c for c in cols]
        geom = torch.cat(cols, dim=-1).to(self.device, torch.float32).contiguous()
        # Polygon.__init__ sorts (cotix/_convex_shapes.py:143-144): do it on the device
        off = 0
        for p in self.scene.parts:
            n = p.geom_floats()
            if isinstance(p, AbstractPolygon) and not p.presorted:
                sl = geom[..., off:off + n].contiguous()
                nv = n // 2
                _ffi.check(_ffi.lib.cotix_order_clockwise(_ffi.ptr(sl), sl.numel() // n, nv,
                                                          _ffi.stream_ptr(self.device)), "cotix_order_clockwise")
                geom[..., off:off + n] = sl
            off += n
        assert off + (4 * len(self.bodies) if self.scene.per_env_params else 0) == self.scene.geom_floats
        return geom

    def polygon_min_angle(self):
        """Smallest interior angle (degrees) of any polygon part of the uploaded
        geometry, over every env (180 when the scene has no polygon; NaN
        geometry gives NaN).  Computed on the geometry's device in float64;
        only the scalar comes back."""
        g = self.geom.detach()
        amin, off = 180.0, 0
        for p in self.scene.parts:
            n = p.geom_floats()
            if isinstance(p, AbstractPolygon):
                v = g[..., off:off + n].to(torch.float64).reshape(*g.shape[:-1], n // 2, 2)
                a, b = v.roll(1, -2) - v, v.roll(-1, -2) - v
                cr = (a[..., 0] * b[..., 1] - a[..., 1] * b[..., 0]).abs()
                m = float(torch.rad2deg(torch.atan2(cr, (a * b).sum(-1))).min())  # torch's min propagates NaN
                amin = m if not (m >= amin) else amin  # NaN sticks
            off += n
        return amin

    def broadphase_ok(self):
        """Informational: every polygon interior angle of the uploaded local
        geometry >= 0.5 degrees.  COTIX_STAGE_BROADPHASE no longer depends on
        it: the kernel checks the conditions of its exactness argument on the
        world shapes of every pair it skips."""
        key = (id(self.geom), self.geom._version)
        if getattr(self, "_bp_key", None) != key:
            self._bp_ok = self.polygon_min_angle() >= 0.5
            self._bp_key = key
        return self._bp_ok

    def _stages(self, stages):
        return stages

    def set_variant(self, envs_per_wave=0, specialize=True):
        """See Scene.set_variant (a tiling choice; results are identical)."""
        self.scene.set_variant(envs_per_wave, specialize)
        return self

    # -- state access -----------------------------------------------------
    def body(self, i):
        return BodyView(self, i)

    def set_dyn(self, dyn):
        self.dyn.copy_(dyn)

    # -- hot path ---------------------------------------------------------
    def step(self, n_steps=1, dt=1e-2, stages=_ffi.STAGES_ROBOCUP, action=None, action_body=0,
             dyn_reset=None, resets=None, trace=None):
        """Fused driver step (examples/test_viz.py:24-44 / :61-69), n_steps times.

        dyn_reset/resets: episode restarts on an error trip (cotix_step_autoreset
        semantics; combinable with `action`).  trace: a dict that receives the
        collider's per-step choices, "chosen" i32 [n_steps, n_bodies, B] (j* of
        body i, cotix/_colliders.py:274-295) and "cells" i32 [n_steps, n_bodies,
        n_bodies, B] (the winning scan candidate of all_contacts[i, j],
        ind1 | ind2 << 9 | type << 18, -1 = empty; :208-268)."""
        s = _ffi.stream_ptr(self.device)
        if action is not None:
            action = action.to(self.device, torch.float32).contiguous()
            if action.shape != (n_steps, self.B, 2):
                raise ValueError("action must be [n_steps, B, 2]")
        if dyn_reset is not None and tuple(dyn_reset.shape) != tuple(self.dyn.shape):
            raise ValueError("dyn_reset must have the state's shape [n_bodies, 6, B]")
        chosen = cells = None
        if trace is not None:
            nb = len(self.bodies)
            chosen = torch.empty(n_steps, nb, self.B, dtype=torch.int32, device=self.device)
            cells = torch.empty(n_steps, nb, nb, self.B, dtype=torch.int32, device=self.device)
            trace["chosen"], trace["cells"] = chosen, cells
        if dyn_reset is None and trace is None:
            _ffi.check(_ffi.lib.cotix_step(
                self.scene.handle, _ffi.ptr(self.dyn), _ffi.ptr(self.keys), _ffi.ptr(self.err),
                _ffi.ptr(self.geom), self.geom_stride, self.B, int(n_steps), float(dt), int(self._stages(stages)),
                _ffi.ptr(action), int(action_body), s), "cotix_step")
            return self
        _ffi.check(_ffi.lib.cotix_step_ex(
            self.scene.handle, _ffi.ptr(self.dyn), _ffi.ptr(self.keys), _ffi.ptr(self.err), _ffi.ptr(self.geom),
            self.geom_stride, self.B, int(n_steps), float(dt), int(self._stages(stages)), _ffi.ptr(action),
            int(action_body), _ffi.ptr(dyn_reset), _ffi.ptr(resets), _ffi.ptr(chosen), _ffi.ptr(cells), s),
            "cotix_step_ex")
        return self

    def step_state(self, dyn, keys, err, n_steps=1, dt=1e-2, stages=_ffi.STAGES_ROBOCUP, action=None,
                   action_body=0):
        """The fused step on caller-owned state tensors (same layouts as
        self.dyn / self.keys / self.err) with this world's scene and geometry."""
        for t, shape in ((dyn, tuple(self.dyn.shape)), (keys, (self.B, 2)), (err, (self.B,))):
            if tuple(t.shape) != shape or not t.is_contiguous() or t.device != self.dyn.device:
                raise ValueError("state tensor shape/device/layout mismatch")
        if action is not None:
            action = action.to(self.device, torch.float32).contiguous()
            if action.shape != (n_steps, self.B, 2):
                raise ValueError("action must be [n_steps, B, 2]")
        _ffi.check(_ffi.lib.cotix_step(
            self.scene.handle, _ffi.ptr(dyn), _ffi.ptr(keys), _ffi.ptr(err), _ffi.ptr(self.geom), self.geom_stride,
            self.B, int(n_steps), float(dt), int(self._stages(stages)), _ffi.ptr(action), int(action_body),
            _ffi.stream_ptr(self.device)), "cotix_step")

    def eval_state(self, dyn, keys, err, n_nfe, wfe, dt, stages, judge=None, control=None, reward=None,
                   finished=None, action=None, action_body=0, reset_mode=0, dyn_reset=None, resets=None, obs=None):
        """cotix_eval on caller-owned state tensors (same layouts as self.dyn /
        self.keys / self.err): AbstractEnvironment.eval's NFE x WFE loop in one
        launch.  judge / control: ctypes cotix_judge / cotix_control (or None);
        action f32 [B, 2] held over the env-steps; reward f32 [B] and finished
        i32 [B] in/out; obs f32 [B, n_bodies, 6] out (nullable)."""
        self.eval_launcher(dyn, keys, err, n_nfe, wfe, dt, stages, judge, control, reward, finished, action,
                           action_body, reset_mode, dyn_reset, resets, obs)()

    def eval_launcher(self, dyn, keys, err, n_nfe, wfe, dt, stages, judge=None, control=None, reward=None,
                      finished=None, action=None, action_body=0, reset_mode=0, dyn_reset=None, resets=None,
                      obs=None):
        """eval_state's launch prepared once: checks every tensor and converts
        every argument now, and returns launch(action=None, stream=None), which
        calls cotix_eval with them on the current stream (or `stream`, a raw
        stream handle) -- the per-step host cost of an RL loop that steps the
        same buffers over and over (BatchedEnv.step).  launch(action=t) swaps
        in another f32 [B, 2] action tensor (shape/dtype/device checked, then
        only its pointer); the returned launcher keeps every tensor alive."""
        for t, shape in ((dyn, tuple(self.dyn.shape)), (keys, (self.B, 2)), (err, (self.B,))):
            if tuple(t.shape) != shape or not t.is_contiguous() or t.device != self.dyn.device:
                raise ValueError("state tensor shape/device/layout mismatch")
        f32, i32 = torch.float32, torch.int32
        for t, shape, dt_ in ((dyn, tuple(self.dyn.shape), f32), (keys, (self.B, 2), i32), (err, (self.B,), i32),
                              (reward, (self.B,), f32), (finished, (self.B,), i32), (action, (self.B, 2), f32),
                              (dyn_reset, tuple(self.dyn.shape), f32), (resets, (self.B,), i32),
                              (obs, (self.B, len(self.bodies), 6), f32)):
            if t is not None and (tuple(t.shape) != shape or not t.is_contiguous() or t.device != self.dyn.device):
                raise ValueError("eval tensor shape/device/layout mismatch")
            if t is not None and t.dtype != dt_:  # the kernel reads f32 / 32-bit words
                raise ValueError("eval tensor dtype %s, expected %s" % (t.dtype, dt_))
        import ctypes
        args = [self.scene.handle, _ffi.ptr(dyn), _ffi.ptr(keys), _ffi.ptr(err), _ffi.ptr(self.geom),
                ctypes.c_int(self.geom_stride), ctypes.c_int(self.B), ctypes.c_int(int(n_nfe)), ctypes.c_int(int(wfe)),
                ctypes.c_float(float(dt)), ctypes.c_int(int(self._stages(stages))),
                None if judge is None else ctypes.pointer(judge), None if control is None else ctypes.pointer(control),
                _ffi.ptr(action), ctypes.c_int(int(action_body)), _ffi.ptr(reward), _ffi.ptr(finished),
                ctypes.c_int(int(reset_mode)), _ffi.ptr(dyn_reset), _ffi.ptr(resets), _ffi.ptr(obs)]
        keep = (dyn, keys, err, self.geom, judge, control, action, reward, finished, dyn_reset, resets, obs)
        fn, dev_index = _ffi.lib.cotix_eval, self.dyn.device.index
        # the current stream at each launch, as every other op (the raw handle without a Stream object)
        raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        cur_stream = raw if raw is not None else (lambda i: torch.cuda.current_stream(i).cuda_stream)
        act_shape, act_dev = (self.B, 2), self.dyn.device

        def launch(action=None, stream=None):
            a = args
            if action is not None:
                if tuple(action.shape) != act_shape or action.dtype != torch.float32 or action.device != act_dev \
                        or not action.is_contiguous():
                    raise ValueError("action must be a contiguous f32 [B, 2] tensor on the world's device")
                a = list(args)
                a[13] = ctypes.c_void_p(action.data_ptr())
            st = cur_stream(dev_index) if stream is None else stream
            rc = fn(*a, ctypes.c_void_p(st))
            if rc != 0:
                _ffi.check(rc, "cotix_eval")
            return keep  # (the launch reads them asynchronously)

        return launch

    # -- body-level operators (UniversalShape, cotix/_universal_shape.py:87-132) --
    def penetrates_with(self, i, j):
        """(collides bool [B], penetration f32 [B, 2]) of body i against body j:
        collides_with over all part pairs, then penetration_depth (EPA, 48 it.)."""
        col = torch.empty(self.B, dtype=torch.int32, device=self.device)
        pen = torch.empty(self.B, 2, dtype=torch.float32, device=self.device)
        _ffi.check(_ffi.lib.cotix_body_penetration(
            self.scene.handle, _ffi.ptr(self.dyn), _ffi.ptr(self.geom), self.geom_stride, self.B, int(i), int(j),
            _ffi.ptr(col), _ffi.ptr(pen), _ffi.stream_ptr(self.device)), "cotix_body_penetration")
        return col.bool(), pen

    def collides_with(self, i, j):
        return self.penetrates_with(i, j)[0]

    def aabb(self, i, err=None):
        """AABB.of of body i (lo.x, lo.y, up.x, up.y) [B, 4]; err bits OR-ed into `err`."""
        out = torch.empty(self.B, 4, dtype=torch.float32, device=self.device)
        _ffi.check(_ffi.lib.cotix_body_aabb(
            self.scene.handle, _ffi.ptr(self.dyn), _ffi.ptr(self.geom), self.geom_stride, self.B, int(i),
            _ffi.ptr(out), _ffi.ptr(err), _ffi.stream_ptr(self.device)), "cotix_body_aabb")
        return out

    def possibly_collides_with(self, i, j):
        """Broadphase: the two bodies' AABBs overlap (the negation of
        aabb_vs_aabb's separation test, cotix/_contacts.py:62-65)."""
        a, b = self.aabb(i), self.aabb(j)
        sep = (a[:, 3] <= b[:, 1]) | (a[:, 2] <= b[:, 0]) | (a[:, 1] >= b[:, 3]) | (a[:, 0] >= b[:, 2])
        return ~sep

    def observe(self, out=None, dyn=None):
        """f32 [B, n_bodies, 6] (px, py, vx, vy, angle, angular_velocity per
        body) from the SoA state, one device transpose (cotix_observe)."""
        d = self.dyn if dyn is None else dyn
        nb = len(self.bodies)
        if out is None:
            out = torch.empty(self.B, nb, 6, dtype=torch.float32, device=self.device)
        _ffi.check(_ffi.lib.cotix_observe(_ffi.ptr(d), nb, self.B, _ffi.ptr(out), _ffi.stream_ptr(self.device)),
                   "cotix_observe")
        return out

    def check_state(self, err=None):
        """class_invariant of the state (cotix/_design_by_contract.py:80-107):
        err |= ERR_STATE_NONFINITE for every env with a NaN/inf state word."""
        e = self.err if err is None else err
        _ffi.check(_ffi.lib.cotix_check_state(_ffi.ptr(self.dyn), len(self.bodies), self.B, _ffi.ptr(e),
                                              _ffi.stream_ptr(self.device)), "cotix_check_state")
        return e

    def euler(self, dt):
        _ffi.check(_ffi.lib.cotix_physics_euler(_ffi.ptr(self.dyn), len(self.bodies), self.B, float(dt),
                                                _ffi.stream_ptr(self.device)), "cotix_physics_euler")
        return self

    def collide(self, keys=None):
        k = self.keys if keys is None else keys.to(self.device, torch.int32).contiguous()
        _ffi.check(_ffi.lib.cotix_collider_resolve(
            self.scene.handle, _ffi.ptr(self.dyn), _ffi.ptr(k), _ffi.ptr(self.err), _ffi.ptr(self.geom),
            self.geom_stride, self.B, _ffi.stream_ptr(self.device)), "cotix_collider_resolve")
        return self

    def lunar_constraints(self):
        _ffi.check(_ffi.lib.cotix_lunar_constraints(_ffi.ptr(self.dyn), self.B, _ffi.stream_ptr(self.device)),
                   "cotix_lunar_constraints")
        return self
