/* cotix_amd.h -- C-ABI of the MI355X-native cotix hot path (libcotix_amd.so).
 *
 * Drop-in boundary for the per-step physics of cotix (DelftMercurians/
 * Parallax).  Plain pointers and sizes only; every float/uint32 pointer
 * argument named "device" is HIP device memory owned by the caller; the
 * library allocates only scene workspace at cotix_scene_create and nothing
 * per step.  Calls are stream-ordered on the given hipStream_t (pass NULL for
 * the default stream); a scene handle is not re-entrant across streams.
 *
 * Return codes: 0 = ok, <0 = error (message in cotix_last_error()).
 *
 * Reference interfaces replaced (file:line in the reference repository):
 *   cotix_step            examples/test_viz.py:24-44 (LunarLander f) and :61-69
 *                         (RoboCup f): Euler -> [gravity] -> collider ->
 *                         [LunarLander.step] -> key = split(key)[0], n_steps times
 *   cotix_step_ex         the same + restarts + actions + the collider's contact
 *                         choices (cotix/_colliders.py:208-295) as a trace
 *   cotix_physics_euler   ExplicitEulerPhysics.step   cotix/_physics_solvers.py:16-33
 *   cotix_collider_resolve RandomizedCollider.resolve cotix/_colliders.py:74-351
 *   cotix_lunar_constraints LunarLander.step          cotix/_lunar_lander.py:145-218
 *   cotix_contacts        _contact_funcs[(Ta,Tb)](a,b) cotix/_colliders.py:21-35,
 *                         cotix/_contacts.py:30-315
 *   cotix_resolve         resolve_collision            cotix/_collision_resolution.py:52-151
 *   cotix_threefry2x32 / cotix_random_split / cotix_random_uniform
 *                         jax.random primitives called at cotix/_colliders.py:142-295
 *   cotix_order_clockwise order_clockwise              cotix/_geometry_utils.py:60-67
 *   cotix_rollout / cotix_rollout_backward  BASELINE config 5
 *   cotix_body_penetration UniversalShape.collides_with / penetrates_with
 *                         cotix/_universal_shape.py:87-132
 *   cotix_body_aabb       UniversalShape.possibly_collides_with (AABB.of of the
 *                         body)  cotix/_universal_shape.py:109-110, _convex_shapes.py:68-77
 *   cotix_observe         the observation tensor of env.step()
 *   cotix_render          env.draw(painter) via Painter callbacks  cotix/_viz.py:55-75,
 *                         cotix/_robocup.py:140-150, cotix/_lunar_lander.py:220-225
 *   cotix_check_state     class_invariant  cotix/_design_by_contract.py:80-107
 *   cotix_eval            AbstractEnvironment.eval     cotix/_envs.py:37-132 with a
 *                         device AbstractJudge (:9-28) / AbstractControl
 *                         (cotix/_controls.py:16-27); also env.step() -> (obs,
 *                         reward, done) of the north star
 */
#ifndef COTIX_AMD_H
#define COTIX_AMD_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cotix_scene cotix_scene;
typedef struct ihipStream_t* cotix_stream_t; /* == hipStream_t */

/* shape registry type ids (exact Python types of cotix/_convex_shapes.py) */
enum {
  COTIX_CIRCLE = 0,
  COTIX_AABB = 1,
  COTIX_POLYGON = 2,
  COTIX_POLYGON3 = 3,
  COTIX_POLYGON4 = 4,
  COTIX_POLYGON5 = 5,
  COTIX_POLYGON6 = 6
};

/* contact function ids (values of the _contact_funcs registry) */
enum {
  COTIX_FN_AABB_AABB = 0,
  COTIX_FN_CIRCLE_CIRCLE = 1,
  COTIX_FN_CIRCLE_AABB = 2,
  COTIX_FN_POLY_POLY = 3,
  COTIX_FN_AABB_POLY = 4,
  COTIX_FN_CIRCLE_POLY = 5
};

/* cotix_step stage bits */
enum {
  COTIX_STAGE_EULER = 1,        /* ExplicitEulerPhysics.step                  */
  COTIX_STAGE_GRAVITY = 2,      /* body 0 velocity += (0, -0.002)  (LL driver) */
  COTIX_STAGE_COLLIDER = 4,     /* RandomizedCollider.resolve(bodies, key)    */
  COTIX_STAGE_LUNAR = 8,        /* LunarLander.step joint constraints          */
  COTIX_STAGE_ADVANCE_KEY = 16, /* key = split(key)[0]                        */
  /* broadphase of the collider's polygon contacts (opt-in, results unchanged):
   * a polygon x polygon / AABB x polygon pair whose world AABBs are separated
   * by more than 2^-8 * S + 2^-16 (S = the pair's largest |coordinate|) and
   * whose world shapes pass the argument's shape conditions (strictly convex,
   * no sharp vertex with sin(angle) < 2^-7: checked by the kernel once per
   * rebuilt world part; no edge of one within 2^-9 of parallel to an edge of
   * the other: checked per pair on the parts' edge pseudo-angles) skips
   * GJK, EPA and the contact points: every term of _contact_from_edges is
   * then provably NaN / false, so the reference's contact is NaN
   * ("Broadphase exactness"). */
  COTIX_STAGE_BROADPHASE = 32,
  COTIX_STAGES_ROBOCUP = 1 | 4 | 16,
  COTIX_STAGES_LUNAR = 1 | 2 | 4 | 8 | 16
};

/* per-env error bits (eqx.error_if sites on the path) */
enum {
  COTIX_ERR_CIRCLE_AABB_CCP = 1, /* cotix/_contacts.py:105-107 */
  COTIX_ERR_AABB_INVALID = 2,    /* AABB.of, cotix/_convex_shapes.py:74-75 (body-level broadphase) */
  COTIX_ERR_STATE_NONFINITE = 4  /* class_invariant, cotix/_design_by_contract.py:80-107: NaN/inf state */
};

/* jax.random threefry layouts (jax/_src/prng.py).  The reference
 * pins no JAX version (pyproject.toml:16): JAX 0.4.x defaults to the legacy
 * layout (jax_threefry_partitionable=False), JAX >= 0.5 to the partitionable
 * one, so the collider's contact choices depend on which JAX runs it.
 *   legacy:        split(k, n)[i] = words 2i, 2i+1 of threefry(k, iota(2n))
 *                  split in halves; random_bits word m of a count-c draw from
 *                  the halves of iota(c) (zero pad when c is odd)
 *   partitionable: split(k, n)[i] = threefry(k, (0, i)); random_bits word m =
 *                  y0 ^ y1 of threefry(k, (0, m)) */
enum { COTIX_PRNG_LEGACY = 0, COTIX_PRNG_PARTITIONABLE = 1 };

/* The reference's hard-coded constants on the hot path, as a scene parameter
 * block (defaults = the reference's literals; cotix_params_default fills them):
 *   prng_layout       COTIX_PRNG_LEGACY        every jax.random call of the step
 *   baumgarte         0.3    cotix/_collision_resolution.py:105 (baumgarte_term)
 *   baumgarte_dt      0.01   :115 (the divisor of the penetration term: "/ dt is missing")
 *   contact_p         0.5    cotix/_colliders.py:220-223 (bernoulli p of a candidate's write)
 *   gjk_max_steps     32     cotix/_collisions.py:101 (GJK while_loop max_steps), >= 0
 *   epa_max_iters     48     cotix/_contacts.py:271,295 (the min(48, ...) cap of
 *                            aabb_vs_polygon / polygon_vs_polygon), >= 3
 *   epa_circle_iters  128    cotix/_contacts.py:162-163 (circle_vs_polygon), 3..128
 *   epa_body_iters    48     cotix/_universal_shape.py:120 (penetration_depth), 3..128
 * The GJK start direction random_direction(PRNGKey(1)) (cotix/_collisions.py:
 * 287-298) follows prng_layout. */
typedef struct cotix_params {
  int prng_layout;
  float baumgarte;
  float baumgarte_dt;
  float contact_p;
  int gjk_max_steps;
  int epa_max_iters;
  int epa_circle_iters;
  int epa_body_iters;
} cotix_params;
int cotix_params_default(cotix_params* out);

/* Compile a scene (the collider's trace-time enumeration, cotix/_colliders.py:86-131).
 *   body_params [n_bodies][4] host: mass, inertia, elasticity, friction_coefficient
 *   part_body   [n_parts]  host: owning body (parts grouped by body, in shape order)
 *   part_type   [n_parts]  host: COTIX_CIRCLE .. COTIX_POLYGON6
 *   part_nverts [n_parts]  host: vertex count for polygons (ignored otherwise)
 * Illegal type pairs are rejected here (the reference raises RuntimeError
 * at trace time, cotix/_colliders.py:103-107). */
int cotix_scene_create(int n_bodies, const float* body_params, int n_parts, const int* part_body,
                       const int* part_type, const int* part_nverts, cotix_scene** out);
/* the same with a parameter block (NULL: the defaults); out-of-range fields
 * are rejected here.  cotix_scene_params returns the scene's block. */
int cotix_scene_create_ex(int n_bodies, const float* body_params, int n_parts, const int* part_body,
                          const int* part_type, const int* part_nverts, const cotix_params* params,
                          cotix_scene** out);
/* cotix_scene_create_ex with flags:
 *   COTIX_SCENE_PER_ENV_BODY_PARAMS  every env carries its own mass, inertia,
 *     elasticity and friction_coefficient per body -- a vmapped pytree whose
 *     parameter leaves vary over the batch (cotix/_bodies.py:140-154,
 *     domain randomization).  They travel in the env's local geometry: the
 *     scene's geometry floats (cotix_scene_geom_floats) are the parts' words
 *     followed by [n_bodies][4] parameter words, per env (geom_stride > 0;
 *     body_params here is a template that only the checks read).  Divisions
 *     by mass and inertia are then IEEE divisions (no scene-time reciprocal)
 *     and the scene runs the generic kernel. */
enum { COTIX_SCENE_PER_ENV_BODY_PARAMS = 1 };
int cotix_scene_create_ex2(int n_bodies, const float* body_params, int n_parts, const int* part_body,
                           const int* part_type, const int* part_nverts, const cotix_params* params, int flags,
                           cotix_scene** out);
int cotix_scene_params(const cotix_scene* scene, cotix_params* out);
int cotix_scene_destroy(cotix_scene* scene);
/* floats of local part geometry the scene expects per env (circle: r,cx,cy,0;
 * AABB: lo.x,lo.y,up.x,up.y; polygon: x,y per vertex), parts in order. */
int cotix_scene_geom_floats(const cotix_scene* scene);
/* introspection for tests: counts of distinct contacts / cells / candidates / type keys */
int cotix_scene_info(const cotix_scene* scene, int* n_contacts, int* n_cells, int* n_candidates, int* n_types);
/* Kernel variant of the scene's launches (no reference counterpart: a tiling
 * choice; every variant computes the same bits).  envs_per_wave: 0 (the
 * scene's default) | 1 | 2 | 4 | 8; specialize: 1 (default) lets the two reference scenes
 * under the default constants use kernels with their whole scene header as a
 * compile-time constant, 0 forces the generic kernel.
 * cotix_scene_variant reports what a step launch uses: the tiling and the
 * specialization id (0 generic, 1 RoboCup, 2 LunarLander, 3 RoboCup and 4
 * LunarLander in the partitionable PRNG layout, 5 the box world's structure:
 * 3 AABB walls and 4 circles, legacy layout).
 * The tiling is a scene property: cotix_scene_create(_ex) sets the default to
 * 4 envs per wave, or the largest of 2 and 1 whose workgroup (the hot tables
 * + 4 wave tiles and scratches) fits the CU's 160 KiB of LDS; a scene whose
 * tiles do not fit four at a time even at one env per wave runs workgroups of
 * 2 or 1 waves (each wave still owns one env's tile; the generic kernel), and
 * cotix_scene_waves_per_group reports the count.  Hard caps: 16 bodies, 32
 * parts, 511 distinct contacts and candidate-list entries, the hot-table and
 * cell limits of the scene compiler, and one env's tile + the tables within
 * 160 KiB -- a scene beyond them is rejected at creation with the reason
 * (the LDS message gives the bytes); cotix_scene_set_variant rejects an
 * explicit tiling that does not fit. */
int cotix_scene_set_variant(cotix_scene* scene, int envs_per_wave, int specialize);
int cotix_scene_variant(const cotix_scene* scene, int* envs_per_wave, int* spec);
int cotix_scene_waves_per_group(const cotix_scene* scene);

/* Fused step, n_steps times, in place.
 *   dyn   device f32 [n_bodies][6][B]  (px, py, vx, vy, angle, angular_velocity)
 *   keys  device u32 [B][2]            collider key per env (advanced when
 *                                      COTIX_STAGE_ADVANCE_KEY is set)
 *   err   device u32 [B]               OR-ed error bits (caller zeroes)
 *   geom  device f32 [geom_floats] (geom_stride == 0, shared by all envs) or
 *                    [B][geom_stride] (per-env geometry, geom_stride >= geom_floats)
 *   action nullable device f32 [n_steps][B][2]: added to the velocity of body
 *          action_body after the Euler stage (differentiable-config hook). */
int cotix_step(cotix_scene* scene, float* dyn, uint32_t* keys, uint32_t* err, const float* geom,
               int geom_stride, int B, int n_steps, float dt, int stages, const float* action,
               int action_body, cotix_stream_t stream);

/* cotix_step with episode restarts: after every env-step, an env whose error
 * bits are set (the reference raises XlaRuntimeError there) is restored from
 *   dyn_reset device f32 [n_bodies][6][B]; its err word is cleared and
 *   resets[env] (device u32 [B], nullable) is incremented.  The key chain
 * continues.  Used by the benchmark to keep a sustained batch. */
int cotix_step_autoreset(cotix_scene* scene, float* dyn, uint32_t* keys, uint32_t* err, const float* geom,
                         int geom_stride, int B, int n_steps, float dt, int stages, const float* dyn_reset,
                         uint32_t* resets, cotix_stream_t stream);

/* The fused step with every option (all pointers nullable):
 *   action [n_steps][B][2]  added to body action_body's velocity after Euler
 *   dyn_reset/resets        episode restarts as cotix_step_autoreset (the
 *                           action keeps applying to a restarted env)
 *   chosen  device i32 [n_steps][n_bodies][B]: the collider's chosen partner
 *           j* of body i at each step (choose_random_contact,
 *           cotix/_colliders.py:274-295; i itself when the body has no
 *           contact; -1 when the collider stage is off)
 *   cells   device i32 [n_steps][n_bodies][n_bodies][B]: for cell (i, j) the
 *           candidate of the reference's scan whose contact all_contacts[i, j]
 *           holds after the scan (the LAST passing one, :208-268), encoded
 *           ind1 | ind2 << 9 | type << 18 (type = index of the (Ta, Tb) key in
 *           dict-insertion order, ind1/ind2 = positions in its two candidate
 *           lists, :86-113); -1 for an empty (NaN) cell or collider stage off.
 * Both traces describe the step BEFORE a restart replaces the state. */
int cotix_step_ex(cotix_scene* scene, float* dyn, uint32_t* keys, uint32_t* err, const float* geom, int geom_stride,
                  int B, int n_steps, float dt, int stages, const float* action, int action_body,
                  const float* dyn_reset, uint32_t* resets, int32_t* chosen, int32_t* cells, cotix_stream_t stream);

/* Device judge: AbstractJudge (cotix/_envs.py:9-28) in the form the step
 * kernel evaluates after every env-step.  s = the env's state words
 * [n_bodies*6] (body-major: px, py, vx, vy, angle, angular_velocity):
 *   judge(s)      = sum_k rate_w[k] * s[k]                       (reward rate)
 *                   (+ piece_r(s) while rate region r is the first rate region
 *                   holding s: piecewise linear, below)
 *   end_reward(s) = sum_k end_w[k] * s[k]  (+ region_reward[r] for the first
 *                   region r that holds s)
 *   is_done(s)    = some region holds s, or (done_on_error and the env's
 *                   error bits are set -- the reference raises there)
 * Sums run in k order over the NONZERO weights (at most 16 each), starting
 * from the first term (none: 0).  Region r holds s when region_lo[r][q] <
 * s[6*region_body[r] + q] < region_hi[r][q] for every q (NaN is never inside;
 * +-inf leaves a word free).
 * cotix_judge and cotix_control must be zero-initialised (`= {0}` or memset)
 * before they are filled: every field is read, including those added after
 * the first layout (the rate regions; saturate / clip_lo / clip_hi).  A
 * saturate other than 0 / 1, a done_on_error other than 0 / 1, a NaN clip
 * bound or a count outside its range is rejected with an error. */
#define COTIX_JUDGE_REGIONS 4
#define COTIX_MAX_STATE_WORDS 96
typedef struct cotix_judge {
  float rate_w[COTIX_MAX_STATE_WORDS];
  float end_w[COTIX_MAX_STATE_WORDS];
  int n_regions;
  int region_body[COTIX_JUDGE_REGIONS];
  float region_lo[COTIX_JUDGE_REGIONS][6];
  float region_hi[COTIX_JUDGE_REGIONS][6];
  float region_reward[COTIX_JUDGE_REGIONS];
  int done_on_error;
  /* piecewise-linear reward rate: n_rate_regions boxes over one body's state
   * (held as the done regions are; they do not end the episode).  While rate
   * region r is the first holding s, piece_r(s) = sum_k rate_region_w[r][k] *
   * s[k] (nonzero weights in k order, from the first term, at most 8) +
   * rate_region_bias[r] (if nonzero) is added: judge(s) = base + piece_r when
   * both have terms, else whichever has one (none: 0) */
  int n_rate_regions;
  int rate_region_body[COTIX_JUDGE_REGIONS];
  float rate_region_lo[COTIX_JUDGE_REGIONS][6];
  float rate_region_hi[COTIX_JUDGE_REGIONS][6];
  float rate_region_w[COTIX_JUDGE_REGIONS][COTIX_MAX_STATE_WORDS];
  float rate_region_bias[COTIX_JUDGE_REGIONS];
} cotix_judge;

/* Device control: AbstractControl (cotix/_controls.py:16-27) whose dense
 * signal is a velocity impulse on `body`, re-evaluated before every env-step
 * from that body's state s[6] and added after Euler (world.forward(state,
 * signal), cotix/_envs.py:72-75):
 *   dv[i] = sum_q gain[i][q] * (target[i][q] - s[q])  (nonzero gains, q order,
 *           from the first term)  + bias[i] (if nonzero)
 * and with saturate != 0 the saturating (clipped) form
 *   dv[i] = clip(dv[i], clip_lo[i], clip_hi[i])  (jnp.clip: min(hi, max(lo, x)),
 *           NaN propagates) */
typedef struct cotix_control {
  int body;
  float gain[2][6];
  float target[2][6];
  float bias[2];
  int saturate;
  float clip_lo[2];
  float clip_hi[2];
} cotix_control;

/* AbstractEnvironment.eval (cotix/_envs.py:37-132) fused into ONE launch:
 * num_NFEs x WFE_scale env-steps (n_steps = n_nfe * wfe, dt per env-step),
 * per env with the reference's carry -- at each NFE start end_reward is taken
 * (unless finished) and is_done checked; after every env-step the first done
 * state becomes the premature out with reward + end_reward; reward +=
 * judge(s) * dt; at the NFE end a done env takes its premature out (state,
 * key, err, reward) and `finished` is set.
 *   judge      nullable host struct (NULL: no reward / done bookkeeping)
 *   control    nullable host struct (NULL: no device control)
 *   action     nullable device f32 [B][2]: a held impulse added to action_body
 *              every env-step after Euler (env.step(action))
 *   reward     device f32 [B] in/out (the carry's reward; zero it for a fresh eval)
 *   finished   device u32 [B] in/out (the carry's flag)
 *   reset_mode 0: none; 2: envs finished at entry restart from dyn_reset
 *              (err, finished cleared, resets[env]++, key chain continues) --
 *              next-step autoreset for env.step() (judge required: it is what
 *              sets and clears `finished`); 1: restart on error bits after
 *              each env-step (cotix_step_autoreset; judge must be NULL)
 *   obs        nullable device f32 [B][n_bodies][6]: the final observation,
 *              written by the same launch */
int cotix_eval(cotix_scene* scene, float* dyn, uint32_t* keys, uint32_t* err, const float* geom, int geom_stride,
               int B, int n_nfe, int wfe, float dt, int stages, const cotix_judge* judge,
               const cotix_control* control, const float* action, int action_body, float* reward,
               uint32_t* finished, int reset_mode, const float* dyn_reset, uint32_t* resets, float* obs,
               cotix_stream_t stream);

/* Differentiable rollout (BASELINE config 5: grad(return)/d(action) through a
 * fused n_steps RoboCup rollout).  The reference has no return or action
 * (cotix/_envs.py:9-28 is abstract); SURVEY 8(d) defines them: action[t] is
 * added to the velocity of body action_body after Euler (where the LL driver
 * adds gravity, examples/test_viz.py:27-31), and
 *   ret[env] += sum_{t=1..n_steps} sum_k ret_weights[k] * state_t[k]
 * over the n_bodies*6 state words (terms with ret_weights[k] == 0 are
 * skipped, so NaN bodies outside the return do not poison it).
 *
 * cotix_rollout runs the forward like cotix_step (no restarts) and saves the
 * state and key before every step: saved_dyn device f32
 * [n_steps][ceil(B/4)][n_bodies*6][4] (env blocks of 4: state word r of env g
 * at [step][g/4][r][g%4], so that a wave's 4 envs save one contiguous run),
 * saved_keys device u32 [n_steps][B][2];
 * ret_weights is HOST f32 [n_bodies*6]; ret device f32 [B] (accumulated).
 *
 * cotix_rollout_backward re-plays every step from the saved state (so each
 * discrete choice -- contacts, RNG draws, branches -- is the forward's) and
 * applies the reverse-mode derivative of the executed branch (jax.grad
 * semantics through the reference's lax.cond branches, balanced ties for
 * max/min/clip).  grad_action device f32 [n_steps][B][2] (nullable),
 * grad_dyn0 device f32 [n_bodies][6][B] (nullable) = d ret / d initial state.
 * Polygon contacts (polygon_vs_polygon, aabb_vs_polygon) are differentiated
 * through EPA's final edge (its supports -- polygon vertices, AABB corners --
 * are argmax choices, i.e. constants) and the included contact_from_edges
 * terms, the polygons' world vertices through the body angle
 * (cotix/_collisions.py:115-273, cotix/_contacts.py:205-315); the LunarLander
 * joint stage through its four impulse pairs (cotix/_lunar_lander.py:176-212).
 * Rejected: scenes with circle x polygon contacts (EPA's circle supports
 * chain through every iteration) and the joint stage on a polygon-free scene.
 * The re-play runs without COTIX_STAGE_BROADPHASE (an exact filter). */
int cotix_rollout(cotix_scene* scene, float* dyn, uint32_t* keys, uint32_t* err, const float* geom, int geom_stride,
                  int B, int n_steps, float dt, int stages, const float* action, int action_body,
                  const float* ret_weights, float* ret, float* saved_dyn, uint32_t* saved_keys,
                  cotix_stream_t stream);
int cotix_rollout_backward(cotix_scene* scene, const float* saved_dyn, const uint32_t* saved_keys, const float* geom,
                           int geom_stride, int B, int n_steps, float dt, int stages, const float* action,
                           int action_body, const float* ret_weights, float* grad_action, float* grad_dyn0,
                           cotix_stream_t stream);
/* The same with the forward's decision tape (no reference counterpart: the
 * saved outcome of the forward's discrete work).  cotix_rollout_ex also writes
 *   tape device u32 [n_steps][ceil(B/4)][cotix_rollout_tape_words(scene)][4]
 *        (nullable; env blocks of 4 as saved_dyn):
 *        per step and body the resolution RandomizedCollider.resolve applied
 *        (cotix/_colliders.py:274-336: the chosen partner j*, the contact of
 *        cell (i, j*)) and, in polygon scenes, the final EPA edge of every
 *        contact EPA ran for (cotix/_collisions.py:115-273); in analytic
 *        scenes each resolution's record (impulse applied or not, the
 *        pre-resolution velocities of its two bodies)
 * and cotix_rollout_backward_ex, given that tape (nullable: the re-play of
 * cotix_rollout_backward), restores those decisions instead of re-running the
 * key splits, the narrowphase, the RNG scan and the choice, and starts the
 * VJP of a GJK/EPA contact from the recorded edge.  The gradients are
 * bit-identical to the re-play's. */
int cotix_rollout_tape_words(const cotix_scene* scene);
int cotix_rollout_ex(cotix_scene* scene, float* dyn, uint32_t* keys, uint32_t* err, const float* geom,
                     int geom_stride, int B, int n_steps, float dt, int stages, const float* action, int action_body,
                     const float* ret_weights, float* ret, float* saved_dyn, uint32_t* saved_keys, uint32_t* tape,
                     cotix_stream_t stream);
int cotix_rollout_backward_ex(cotix_scene* scene, const float* saved_dyn, const uint32_t* saved_keys,
                              const uint32_t* tape, const float* geom, int geom_stride, int B, int n_steps, float dt,
                              int stages, const float* action, int action_body, const float* ret_weights,
                              float* grad_action, float* grad_dyn0, cotix_stream_t stream);

/* Body-level operators (UniversalShape, cotix/_universal_shape.py:87-132), per env:
 * cotix_body_penetration: collides_with (GJK over every part pair of the two
 *   bodies, first colliding pair kept, :87-107) and penetrates_with /
 *   penetration_depth (EPA, 48 iterations, :112-132).  Supports are the
 *   reference's wrap_local_support (:32-45, which discards the inverse-rotated
 *   direction).  collides device i32 [B], pen device f32 [B][2] (0 when not
 *   colliding).
 * cotix_body_aabb: AABB.of (cotix/_convex_shapes.py:68-77) of the whole body via
 *   its global support (:47-59) -- a working version of the reference's
 *   possibly_collides_with broadphase (:109-110), whose AABB.of_universal does
 *   not exist.  aabb device f32 [B][4] = lo.x, lo.y, up.x, up.y; err (nullable)
 *   |= COTIX_ERR_AABB_INVALID when x_max <= x_min or y_max <= y_min (the
 *   eqx.error_if, EQX_ON_ERROR=nan: the bound becomes NaN). */
int cotix_body_penetration(const cotix_scene* scene, const float* dyn, const float* geom, int geom_stride, int B,
                           int body_a, int body_b, int* collides, float* pen, cotix_stream_t stream);
int cotix_body_aabb(const cotix_scene* scene, const float* dyn, const float* geom, int geom_stride, int B, int body,
                    float* aabb, uint32_t* err, cotix_stream_t stream);

/* Observation export: obs device f32 [B][n_bodies][6] (per env: px, py, vx,
 * vy, angle, angular_velocity of every body) from dyn [n_bodies][6][B] -- the
 * tensor env.step() returns and the multi-GPU path all-gathers. */
int cotix_observe(const float* dyn, int n_bodies, int B, float* obs, cotix_stream_t stream);

/* Render export (replaces the Painter host callbacks of env.draw(painter),
 * cotix/_viz.py:55-75, cotix/_robocup.py:140-150, cotix/_lunar_lander.py:220-225):
 * prims device f32 [B][cotix_render_count(scene)][4]; per part in scene order:
 * Circle -> (cx, cy, r, NaN), AABB -> its 4 edges, Polygon -> its n edges
 * (x0, y0, x1, y1), of the part transformed by its body (get_edges order). */
int cotix_render_count(const cotix_scene* scene);
int cotix_render(const cotix_scene* scene, const float* dyn, const float* geom, int geom_stride, int B, float* prims,
                 cotix_stream_t stream);

/* Contract check (class_invariant, cotix/_design_by_contract.py:80-107, on the
 * world state): err[env] |= COTIX_ERR_STATE_NONFINITE when any dynamic state
 * word of the env is NaN or infinite.  err device u32 [B]. */
int cotix_check_state(const float* dyn, int n_bodies, int B, uint32_t* err, cotix_stream_t stream);

/* Operator-level entry points (batched over n independent items). */
int cotix_physics_euler(float* dyn, int n_bodies, int B, float dt, cotix_stream_t stream);
int cotix_collider_resolve(cotix_scene* scene, float* dyn, const uint32_t* keys, uint32_t* err,
                           const float* geom, int geom_stride, int B, cotix_stream_t stream);
int cotix_lunar_constraints(float* dyn, int B, cotix_stream_t stream);
/* shapes a, b: device f32 [n][18] = (kind, nverts, d[16]); out device f32
 * [n][4] = (pen.x, pen.y, cp.x, cp.y); err device u32 [n] (may be NULL). */
int cotix_contacts(int fn, int n, const float* a, const float* b, float* out, uint32_t* err,
                   cotix_stream_t stream);
/* dyn1/dyn2 device f32 [n][6] updated in place; par1/par2 [n][4]; contact [n][4] */
int cotix_resolve(int n, float* dyn1, const float* par1, float* dyn2, const float* par2,
                  const float* contact, cotix_stream_t stream);
/* threefry2x32-20 block: out[i] = threefry(keys[i], ctr[i]) (all device u32 [n][2]) */
int cotix_threefry2x32(const uint32_t* keys, const uint32_t* ctr, uint32_t* out, int n,
                       cotix_stream_t stream);
/* out [n][num][2] = jax.random.split(keys[i], num) */
int cotix_random_split(const uint32_t* keys, int n, int num, uint32_t* out, cotix_stream_t stream);
/* out [n][count] = jax.random.uniform(keys[i], (count,), lo, hi) (f32) */
int cotix_random_uniform(const uint32_t* keys, int n, int count, float lo, float hi, float* out,
                         cotix_stream_t stream);
/* The operators above with a parameter block (NULL: the defaults):
 * cotix_contacts_ex  the polygon contacts' GJK steps / EPA iterations and the
 *                    GJK start direction (prng_layout) of `params`
 * cotix_resolve_ex   resolve_collision with its baumgarte / baumgarte_dt
 * cotix_random_split_ex / cotix_random_uniform_ex  in layout COTIX_PRNG_* */
int cotix_contacts_ex(int fn, int n, const float* a, const float* b, float* out, uint32_t* err,
                      const cotix_params* params, cotix_stream_t stream);
int cotix_resolve_ex(int n, float* dyn1, const float* par1, float* dyn2, const float* par2, const float* contact,
                     const cotix_params* params, cotix_stream_t stream);
int cotix_random_split_ex(const uint32_t* keys, int n, int num, int layout, uint32_t* out, cotix_stream_t stream);
int cotix_random_uniform_ex(const uint32_t* keys, int n, int count, float lo, float hi, int layout, float* out,
                            cotix_stream_t stream);

/* GJK and EPA as operators (cotix/_collisions.py:277-329) over the shape rows
 * of cotix_contacts (device f32 [n][18]: kind 0 circle / 1 AABB / 2 polygon,
 * vertex count, geometry); the Minkowski difference is support(a, d) -
 * support(b, -d) (minkowski_diff, cotix/_geometry_utils.py:49-57).
 * cotix_gjk = check_for_collision_convex(a.get_support, b.get_support) with
 *   its default start direction random_direction(PRNGKey(1)) (:287-298; the
 *   layout and gjk_max_steps of `params`, NULL: defaults): hit device i32 [n];
 *   simplex device f32 [n][3][2] -- NaN * simplex when there is no collision
 *   (:300-310).
 * cotix_epa = compute_penetration_vector_convex(a.get_support, b.get_support,
 *   simplex, iters) (:313-329; _get_closest_minkowski_diff :115-273): simplex
 *   device f32 [n][3][2], pen device f32 [n][2]; iters in 3..128 (the
 *   reference's error_if rejects < 3, :130-135). */
int cotix_gjk(int n, const float* a, const float* b, int32_t* hit, float* simplex, const cotix_params* params,
              cotix_stream_t stream);
/* cotix_gjk_ex = check_for_collision_convex(a.get_support, b.get_support,
 *   initial_direction, key) (cotix/_collisions.py:277-298), both nullable:
 *   initial_direction device f32 [n][2] (NULL: the default [nan, nan] for
 *   every item), keys device u32 [n][2] (NULL: PRNGKey(1) for every item).
 *   The start direction is rnd = random_direction(key) (x / |x|, x =
 *   normal(key, (2,)) in the layout of `params`; XLA's f32 ErfInv with a
 *   correctly rounded log1p -- PRNGKey(1) gives the constant of cotix_gjk,
 *   DESIGN.md section 4), then rnd where initial_direction has a NaN, else
 *   rnd * 0.1 + initial_direction * 0.9. */
int cotix_gjk_ex(int n, const float* a, const float* b, const float* initial_direction, const uint32_t* keys,
                 int32_t* hit, float* simplex, const cotix_params* params, cotix_stream_t stream);
int cotix_epa(int n, const float* a, const float* b, const float* simplex, int iters, float* pen,
              cotix_stream_t stream);

/* polygons xy device f32 [n][nverts][2] sorted in place (order_clockwise) */
int cotix_order_clockwise(float* xy, int n, int nverts, cotix_stream_t stream);

const char* cotix_last_error(void);
const char* cotix_version(void);

#ifdef __cplusplus
}
#endif
#endif /* COTIX_AMD_H */
