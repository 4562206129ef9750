/*
 * brax_amd — C ABI of the MI355X-native PBD rigid-body stepper.
 *
 * This is the drop-in boundary for the reference's hot path:
 * what `brax.System.step`, `brax.System.default_qp/info` and the
 * `Env.step/reset` + Episode/AutoReset wrapper stack compute under `jax.jit`
 * is exported here as stream-ordered C calls on caller-owned device buffers.
 *
 *   reference interface                                  replaced by
 *   brax.System(config)          system.py:53-84         bx_system_create
 *   System.step(qp, act)         system.py:244-325       bx_system_step
 *   System.default_qp(a, v)      system.py:112-242       bx_system_default_qp
 *   System.info(qp)              system.py:249-252,327-340  bx_system_info
 *   Env.step + EpisodeWrapper + AutoResetWrapper
 *     ant.py:222-255, wrappers.py:105-148                bx_env_step
 *   Env.reset (+ EpisodeWrapper/AutoResetWrapper.reset counters)
 *     ant.py:198-220, humanoid.py:223-244,
 *     half_cheetah.py:164-180, wrappers.py:94-97,128-133 bx_env_reset
 *   Joint.angle_vel              joints.py:197-226       bx_system_joint_angles
 *
 * Conventions
 *   - Every array argument is a raw device pointer (HBM) owned by the caller.
 *     Sizes are explicit (n_envs, strides in elements); no torch types.
 *   - fp32 throughout on the device (what jit computes; `config.proto` floats
 *     are fp32). The descriptor is float64/int32 host memory, copied at create.
 *   - All calls enqueue on `stream` (a hipStream_t; NULL = default stream) and
 *     return immediately. Not re-entrant per handle.
 *   - Return 0 on success, non-zero on error; `bx_last_error()` returns a
 *     thread-local message. Descriptor errors surface at create time.
 */
#ifndef BRAX_AMD_H_
#define BRAX_AMD_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BX_ABI_VERSION 13

/* joint kinds, actuator kinds, contact functions (descriptor enums) */
enum { BX_JOINT_REVOLUTE = 1, BX_JOINT_UNIVERSAL = 2, BX_JOINT_SPHERICAL = 3 };
/* dynamics modes (config.proto dynamics_mode; system.py:244-247) */
enum { BX_DYN_PBD = 0, BX_DYN_LEGACY_SPRING = 1 };
enum { BX_ACT_TORQUE = 0, BX_ACT_ANGLE = 1 };
enum { BX_COL_CAPSULE_PLANE = 0, BX_COL_CAPSULE_CAPSULE = 1,
       /* box corner vs height map (colliders.py:699-739), capsule end vs
        * clipped plane (:762-802), capsule vs one triangle of a box / mesh
        * (:822-848) */
       BX_COL_HEIGHTMAP = 2, BX_COL_CLIPPED_PLANE = 3, BX_COL_CAPSULE_MESH = 4,
       /* box vs box by the separating axis test (:851-888), 4 rows a pair */
       BX_COL_HULL_HULL = 5 };
enum { BX_FORCE_THRUSTER = 0, BX_FORCE_TWISTER = 1 };
/* env layer kinds (obs / reward programs) */
enum { BX_ENV_NONE = 0, BX_ENV_ANT = 1, BX_ENV_HUMANOID = 2, BX_ENV_HALFCHEETAH = 3,
       BX_ENV_HUMANOID_STANDUP = 4,
       /* the planar walkers (hopper.py:183-246, walker2d.py:194-253): one
        * program, their own constructor defaults */
       BX_ENV_HOPPER = 5, BX_ENV_WALKER2D = 6,
       /* inverted_pendulum.py:133-164, inverted_double_pendulum.py:140-184,
        * acrobot.py:56-95 */
       BX_ENV_INVERTED_PENDULUM = 7, BX_ENV_INVERTED_DOUBLE_PENDULUM = 8, BX_ENV_ACROBOT = 9,
       /* reacher.py:172-236, reacherangle.py:60-106, swimmer.py:216-283,
        * pusher.py:211-242 */
       BX_ENV_REACHER = 10, BX_ENV_REACHERANGLE = 11, BX_ENV_SWIMMER = 12, BX_ENV_PUSHER = 13,
       /* egocentric target envs (ur5e.py:59-135, fetch.py:58-134) */
       BX_ENV_UR5E = 14, BX_ENV_FETCH = 15,
       /* a hand grasping an object (grasp.py:29-190) */
       BX_ENV_GRASP = 16 };
/* observation options. BX_OBS_XY: exclude_current_positions_from_observation
 * = False, the torso's x (and y) precede its z (ant.py:262-265,
 * humanoid.py:289-292: x, y; half_cheetah.py:206-209: x) */
enum { BX_OBS_XY = 1 };

/*
 * System descriptor: the compiled constant arrays of `brax.System`
 * (bodies.py:38-44, joints.py:36-77, actuators.py:28-35, colliders.py:95-114,
 * geometry.py:78-99,242-288, integrators.py:32-48). Built on the host by
 * brax_amd/compiler.py. Shapes in brackets; row-major; J = n_joints etc.
 */
typedef struct bx_desc {
  int32_t n_bodies, n_joints, n_actuators, n_rows, n_groups;
  int32_t substeps, action_size, num_joint_dof;
  double dt, h;
  double gravity[3];
  double velocity_damping, angular_damping;
  /* bodies */
  const double* body_mass;         /* [N] */
  const double* body_inv_inertia;  /* [N,3]  (inverse, body-frame diagonal) */
  const double* pos_mask;          /* [N,3] */
  const double* rot_mask;          /* [N,3] */
  const double* quat_mask;         /* [N,4] */
  /* joints, in application order (grouped by dof like joints.get) */
  const int32_t* joint_type;       /* [J] BX_JOINT_* */
  const int32_t* joint_dof;        /* [J] 1..3 (limit rows in use) */
  const int32_t* joint_free_dofs;  /* [J] -1 for revolute groups */
  const int32_t* joint_body_p;     /* [J] */
  const int32_t* joint_body_c;     /* [J] */
  const int32_t* joint_group;      /* [J] */
  const double* joint_off_p;       /* [J,3] */
  const double* joint_off_c;       /* [J,3] */
  const double* joint_axis_p;      /* [J,3,3] */
  const double* joint_axis_c;      /* [J,3,3] */
  const double* joint_limit;       /* [J,3,2] radians */
  const double* joint_damping;     /* [J] */
  const double* joint_scale_pos;   /* [J] */
  const double* joint_scale_ang;   /* [J] */
  /* actuators, in application order (sorted by type, dof) */
  const int32_t* act_type;         /* [K] BX_ACT_* */
  const int32_t* act_joint;        /* [K] index into joints */
  const int32_t* act_index;        /* [K,3] action index, -1 = masked */
  const int32_t* act_group;        /* [K] */
  const double* act_strength;      /* [K] */
  /* collider groups and flattened contact rows */
  const int32_t* col_oneway;       /* [G] 1 = OneWayCollider */
  const int32_t* col_fn;           /* [G] BX_COL_* */
  const double* col_scale;         /* [G] solver_scale_collide */
  const double* col_velocity_threshold; /* [G] */
  const double* col_baumgarte_erp; /* [G] */
  const int32_t* row_group;        /* [R] */
  const int32_t* row_body_a;       /* [R] */
  const int32_t* row_body_b;       /* [R] */
  const double* row_a_pos;         /* [R,3] collidable offset of a */
  const double* row_a_end;         /* [R,3] capsule end (plane: end point in body a) */
  const double* row_a_radius;      /* [R] */
  const double* row_b_pos;         /* [R,3] */
  const double* row_b_end;         /* [R,3] */
  const double* row_b_radius;      /* [R] */
  const double* row_friction;      /* [R] friction_a * friction_b */
  const double* row_elasticity;    /* [R] */
  /* forces (forces.py:27-138), in application order: Thrusters, then
   * Twisters, each in config order; action indices assigned in config order
   * after the actuators' (post-sphericalisation) dofs */
  int32_t n_forces;
  const int32_t* force_type;       /* [NF] BX_FORCE_* */
  const int32_t* force_body;       /* [NF] */
  const int32_t* force_index;      /* [NF,3] action index (clipped like jp.take) */
  const double* force_strength;    /* [NF] */
  /* NearNeighbors culling (colliders.py:55-89): per group the number of rows
   * kept each step (0 = Pairs, every row active); per row its cell i*U+j in
   * the candidate matrix (-1 for Pairs rows). A culled group's rows are its
   * allowed cells in flat order; Info carries `cutoff` rows for it, nearest
   * first (top_k order). */
  const int32_t* col_cutoff;       /* [G] */
  const int32_t* row_flat;         /* [R] */
  /* legacy_spring dynamics (system.py:342-390, spring_joints.py): joints are
   * springy Revolute / Universal / Spherical groups by dof (no
   * sphericalisation), constrained at the acceleration level; contacts use
   * the impulse model with Baumgarte stabilisation every substep. The three
   * arrays may be NULL for pbd systems. */
  int32_t dynamics_mode;           /* BX_DYN_* */
  const double* joint_stiffness;       /* [J] */
  const double* joint_spring_damping;  /* [J] (default: 0.5 or 2 x sqrt(stiffness)) */
  const double* joint_limit_strength;  /* [J] (default: stiffness) */
  /* extended contact functions: per-row constants (may be NULL when no row
   * uses them)
   *   HEIGHTMAP:     ext[0] cell size; row_hm (offset into hm_data, mesh size)
   *   CLIPPED_PLANE: ext normal 0..2, x 3..5, y 6..8, position 9..11,
   *                  half sizes 12, 13 (b's body frame)
   *   CAPSULE_MESH:  ext triangle p0 0..2, p1 3..5, p2 6..8, normal 9..11
   *                  (b's body frame, winding fixed as geometry.py:138-154) */
  const double* row_ext;           /* [R,16] */
  const int32_t* row_hm;           /* [R,2] */
  int32_t n_hm;
  const double* hm_data;           /* [n_hm] row-major square grids */
  /* HULL_HULL rows: ext (hull a, hull b, contact e) into these box hulls
   * (geometry.py:201-206), body frame */
  int32_t n_hull;
  const double* hull_vert;         /* [H,8,3] corners */
  const double* hull_face;         /* [H,6,4,3] quads, winding fixed */
  const double* hull_norm;         /* [H,6,3] face normals */
  /* NearNeighbors with more `cutoff` than allowed cells: top_k of the
   * masked (-inf) cells picks the lowest flat indices (jax.lax.top_k keeps
   * ties in index order), so those cells are rows too, flagged 1 here; they
   * rank after every allowed cell, in flat order (colliders.py:78-85).
   * NULL = no masked rows. */
  const int32_t* row_nn_masked;    /* [R] */
} bx_desc;

/*
 * Reset descriptor (`System.default_qp`, system.py:112-242; bodies.min_z
 * bodies.py:62-98): joint-tree forward kinematics in depth order, then lift
 * every free root tree so its lowest collider touches z = 0.
 */
typedef struct bx_reset_desc {
  int32_t n_fk;                    /* joints in depth order */
  const int32_t* fk_body_p;        /* [n_fk] */
  const int32_t* fk_body_c;        /* [n_fk] */
  const int32_t* fk_dof_index;     /* [n_fk,3] index into joint angle vector, -1 = 0 */
  const double* fk_rot;            /* [n_fk,4] euler_to_quat(rotation) */
  const double* fk_ref;            /* [n_fk,4] euler_to_quat(reference_rotation) */
  const double* fk_off_p;          /* [n_fk,3] */
  const double* fk_off_c;          /* [n_fk,3] */
  const double* base_qp;           /* [N,13] config default qps (else identity) */
  int32_t n_zpts;                  /* min_z candidate points */
  const int32_t* zpt_body;         /* [n_zpts] */
  const double* zpt_local;         /* [n_zpts,3] point in body frame */
  const double* zpt_radius;        /* [n_zpts] */
  const int32_t* body_zero_cand;   /* [N] 1: min_z also sees 0.0 (plane/none) */
  const int32_t* body_root_group;  /* [N] lift group, -1 = not lifted */
  int32_t n_root_groups;
  /* System.default_angle (system.py:86-110) of this default: the joint-angle
   * vector that bx_env_reset adds its noise to */
  const double* default_angle;     /* [num_joint_dof] */
} bx_reset_desc;

/* A strided view of one fp32 QP field: element (env e, body b, k) lives at
 * ptr[e*env_stride + b*body_stride + k]. Lets the caller pass the reference's
 * (B,N,3)/(B,N,4) arrays or the packed (B,N,16) layout without copies. */
typedef struct bx_field {
  float* ptr;
  int64_t env_stride;
  int64_t body_stride;
} bx_field;

typedef struct bx_qp {
  bx_field pos, rot, vel, ang;     /* rot is wxyz */
} bx_qp;

/* Optional Info outputs of System.step (base.py:136-153); NULL ptr = skip. */
typedef struct bx_info {
  bx_field contact_vel, contact_ang;     /* (B,N,3) accumulated contact P */
  bx_field actuator_vel, actuator_ang;  /* (B,N,3) */
  float* contact_pos;                   /* (B,R,3) contiguous */
  float* contact_normal;                /* (B,R,3) */
  float* contact_penetration;           /* (B,R)   */
  bx_field joint_vel, joint_ang;        /* (B,N,3) accumulated joint P
                                           (legacy_spring; zero under pbd) */
  /* (B,R) contiguous, bx_system_step only (ABI 9): the NearNeighbors cell
   * i * U + j behind each Info contact row, i.e. the `idx` of
   * `jp.top_k(sim.ravel(), cutoff)` in colliders.py:84 for a culled group's
   * rows (nearest first), -1 for Pairs rows */
  int32_t* contact_cell;
} bx_info;

/* Env-layer state of one batch (ant.py:198-255, wrappers.py:83-148).
 * obs (B,O), reward/done/steps/truncation (B,), metrics (B,M); contiguous. */
typedef struct bx_env_state {
  bx_qp qp;
  float* obs;
  float* reward;
  float* done;
  float* metrics;
  float* steps;
  float* truncation;
  /* per-env random stream of the target envs (UR5E, FETCH: the teleported
   * target, ur5e.py:107-113); read from the input state, advanced in the
   * output; NULL for the other kinds */
  uint32_t* rng;
} bx_env_state;

typedef struct bx_env_params {
  int32_t kind;             /* BX_ENV_* */
  int32_t obs_size;
  int32_t n_metrics;
  int32_t episode_length;   /* <= 0: no EpisodeWrapper */
  int32_t action_repeat;    /* EpisodeWrapper action_repeat (>= 1) */
  int32_t auto_reset;       /* AutoResetWrapper present */
  int32_t obs_flags;        /* BX_OBS_* */
  /* env constructor arguments (ant.py:173-183, humanoid.py:196-212,
   * half_cheetah.py:147-158):
   *   ANT:         forward_w(unused=1), ctrl_cost_weight, contact_cost_weight,
   *                healthy_reward, healthy_z_min, healthy_z_max,
   *                terminate_when_unhealthy, use_contact_forces
   *   HUMANOID:    forward_reward_weight, ctrl_cost_weight, 0, healthy_reward,
   *                healthy_z_min, healthy_z_max, terminate_when_unhealthy, 0
   *   HALFCHEETAH: forward_reward_weight, ctrl_cost_weight, 0...
   *   HOPPER / WALKER2D: forward_reward_weight, ctrl_cost_weight,
   *                healthy_reward, healthy_z_min, healthy_z_max (+inf: pass
   *                FLT_MAX), healthy_angle_min, healthy_angle_max,
   *                terminate_when_unhealthy
   *   INVERTED_PENDULUM, INVERTED_DOUBLE_PENDULUM, ACROBOT: none (the
   *                reference envs take no reward arguments)
   *   REACHER:     target body, arm body (indices as floats)
   *   REACHERANGLE: target body, arm body, then per action i (<= 2) the
   *                angle-limit min (coef[2 + i]) and range (coef[4 + i]) the
   *                [-1, 1] action maps onto
   *   SWIMMER:     forward_reward_weight, ctrl_cost_weight, spherical drag,
   *                capsule drag corrections x, y, z (swimmer.py:177-193)
   *   PUSHER:      tip body, object body, goal body
   *   UR5E / FETCH: torso body, target body, target radius, target
   *                distance, target height (a hit target moves to a fresh
   *                random spot on the ring [radius, radius + distance))
   *   GRASP:       palm body, object body, target body, hand body (thumb
   *                proximal), target radius, distance, height */
  float coef[8];
  /* AutoReset targets (first_qp / first_obs); required when auto_reset */
  bx_qp first_qp;
  const float* first_obs;
  /* GRASP: device array [2, A] of per-action (min, range); System.step reads
   * min + range * (a + 1) / 2 (grasp.py:42-52,65); NULL for the other kinds */
  const float* act_map;
} bx_env_params;

typedef struct bx_system bx_system;

int bx_abi_version(void);
const char* bx_last_error(void);
int bx_device_count(int* count);

int bx_system_create(const bx_desc* desc, const bx_reset_desc* reset,
                     int device, bx_system** out);
int bx_system_destroy(bx_system* sys);

/* Threads that own one env in this system's step kernels: 16/32/64 lanes of
 * one wavefront, or a whole 128/256-thread workgroup for large scenes. */
int bx_system_lanes(bx_system* sys);

/* Threads per env of this system's Env.step / rollout kernels (bx_env_step,
 * bx_env_rollout_*): the step kernels' lanes. (ABI 12's opt-in 32-lane
 * spherical joint halves measured slower and were removed in ABI 13.) */
int bx_system_env_lanes(bx_system* sys);

/* The host half of bx_system_create, without a device: the kernel plan the
 * descriptor compiles to -- mode (1 SINGLE: register-hoisted, one env per
 * 16/32/64 lanes; 3 MULTI: one env per 256-thread workgroup; 0 item loops),
 * threads per env, and the System.step kernel's LDS bytes per workgroup
 * (160 KB per CU / that = envs a CU holds at once). */
int bx_system_plan(const bx_desc* desc, const bx_reset_desc* reset, int32_t* mode,
                   int32_t* lanes, int32_t* lds_bytes);

/* LDS bytes per workgroup of this system's System.step kernel (the current
 * variant): with 160 KB per CU it sets how many envs a CU holds at once (the
 * large-scene kernel runs one env per 256-thread workgroup). A diagnostic
 * query; 0 for a null handle. */
int bx_system_lds_bytes(bx_system* sys);

/* Select the register-hoisted kernel variant (default when the system fits:
 * every lane owns <= 1 body/joint/actuator/contact row) or the generic
 * item-loop variant (on = 0). For testing both paths on one system. */
int bx_system_set_single(bx_system* sys, int on);

/* Kernel variant: threads per env (16/32/64/128/256) and constant placement
 * (0: read from HBM in the loops, 1: hoisted to registers, needs <= 1 item per
 * lane, 2: staged in LDS once per workgroup, 3: MULTI, the large-scene pbd
 * kernel at 256 threads: items and <= 4 contact rows per lane hoisted to
 * registers, per-body contact sums through gather tasks). */
int bx_system_set_variant(bx_system* sys, int lanes, int mode);

/* Threads per workgroup of the step kernels: a multiple of the lanes per env,
 * at most 64 (default 64, i.e. 64 / lanes envs per wavefront). Fewer envs per
 * wave means more waves for the same batch (32: two waves per SIMD at 4096
 * Ant envs). Results are identical bit for bit. */
int bx_system_set_block(bx_system* sys, int threads);

/* Physics only: B independent System.step calls (system.py:244-325).
 * act: (B, act_width) with row stride act_stride (0 broadcasts one row).
 * Action indices are clipped to [0, act_width) like the reference's
 * `jp.take(act, index)` (jumpy.py:146-151); act_width >= 1 unless the system
 * reads no action. qp_in and qp_out may not alias. info may be NULL. */
int bx_system_step(bx_system* sys, int64_t n_envs, const bx_qp* qp_in,
                   const float* act, int64_t act_stride, int64_t act_width,
                   const bx_qp* qp_out, const bx_info* info, void* stream);

/* Env layer fused with physics: for each env, EpisodeWrapper-repeat
 * action_repeat times (System.step + obs/reward/done/metrics), then the
 * episode counters and the AutoReset select. in/out may not alias. */
int bx_env_step(bx_system* sys, const bx_env_params* env, int64_t n_envs,
                const bx_env_state* in, const float* act, int64_t act_stride,
                int64_t act_width, const bx_env_state* out, void* stream);

/* bx_env_step on the packed layout, every pointer plain: the input state is
 * qp_in (B,N,16) (pos 0:3, rot 3:7, vel 7:10, ang 10:13), done_in (B,),
 * steps_in (B,) or NULL, rng_in (B,) or NULL; the output is ONE buffer
 * `out` holding qp (B,N,16) | obs (B,O) | reward | done | steps |
 * truncation (B each) | metrics (B,M), and rng_out (B,) or NULL. Same
 * semantics and errors as bx_env_step; the host-side fast path of
 * Env.step. */
int bx_env_step_packed(bx_system* sys, const bx_env_params* env, int64_t n_envs,
                       const float* qp_in, const float* done_in, const float* steps_in,
                       const uint32_t* rng_in, const float* act, int64_t act_stride,
                       int64_t act_width, float* out, uint32_t* rng_out, void* stream);

/* n_steps consecutive bx_env_step_packed calls in ONE launch: an open-loop
 * rollout (the reference's `jax.lax.scan` of `env.step`, e.g.
 * training/acting.py:53-77 generate_unroll, with the actions known up front:
 * random-action rollouts). Step t reads its action rows at act + t *
 * act_step_stride (row stride act_stride) and writes its whole output - qp
 * (B,N,16) | obs (B,O) | reward | done | steps | truncation (B each) |
 * metrics (B,M) - as block t of `out` (block = B * (N*16 + O + 4 + M)
 * floats), its rng stream (target envs) at rng_out + t * B; its input state
 * is step t - 1's output (step 0: qp_in, done_in, steps_in, rng_in). Every
 * step's outputs are bit-identical to the chained single-step calls; the
 * state stays on chip between steps (ABI 9). */
int bx_env_rollout_packed(bx_system* sys, const bx_env_params* env, int64_t n_envs,
                          int32_t n_steps, const float* qp_in, const float* done_in,
                          const float* steps_in, const uint32_t* rng_in, const float* act,
                          int64_t act_stride, int64_t act_step_stride, int64_t act_width,
                          float* out, uint32_t* rng_out, void* stream);

/* bx_env_rollout_packed with the actions drawn on the device inside the same
 * launch: the reference's random-action rollout, a `lax.scan` of `env.step`
 * on `jax.random.uniform` actions (notebooks/environments.ipynb:386-423, the
 * published benchmark loop; the scan of training/acting.py:53-77). Step t's
 * action a of env e is uniform_at(seed, offset + t * step_stride +
 * e * act_width + a) in [lo, hi): the same bits bx_uniform_slabs(act, B * A,
 * K, seed, offset, step_stride, NULL, 0, lo, hi) writes, so this equals that
 * draw followed by bx_env_rollout_packed on its slabs. act_out (optional,
 * (K, n_envs, act_width) contiguous) records the drawn actions. The whole
 * action row is staged on chip: act_width must not exceed the widest row the
 * system reads (every env's own action size fits). Env kinds whose program
 * reads the raw row itself (ReacherAngle, Swimmer, Grasp, Humanoid,
 * HumanoidStandup) are refused: draw with bx_uniform_slabs. n_steps = 0
 * only checks the arguments (ABI 10). */
int bx_env_rollout_random(bx_system* sys, const bx_env_params* env, int64_t n_envs,
                          int32_t n_steps, const float* qp_in, const float* done_in,
                          const float* steps_in, const uint32_t* rng_in, uint64_t seed,
                          uint64_t offset, uint64_t step_stride, float lo, float hi,
                          int64_t act_width, float* act_out, float* out, uint32_t* rng_out,
                          void* stream);

/* Batched System.default_qp from per-env joint angles/velocities
 * (B, num_joint_dof) contiguous (system.py:112-242). */
int bx_system_default_qp(bx_system* sys, int64_t n_envs,
                         const float* joint_angle, const float* joint_velocity,
                         const bx_qp* qp_out, void* stream);

/* Batched reset-time Info (`_pbd_info`, system.py:327-340: Collider.apply). */
int bx_system_info(bx_system* sys, int64_t n_envs, const bx_qp* qp,
                   const bx_info* info, void* stream);

/* Observation and metric widths the env layer writes for `env` on this
 * system (obs_size / n_metrics in bx_env_params must equal them). */
int bx_env_sizes(bx_system* sys, const bx_env_params* env, int32_t* obs_size,
                 int32_t* n_metrics);

/* Env.reset of every env kind, batched, in two launches (ant.py:198-220,
 * humanoid.py:223-244, half_cheetah.py:164-180, humanoid_standup.py:216-230,
 * reacher.py:156-174, reacherangle.py:44-60, pusher.py:178-209,
 * ur5e.py:41-58, fetch.py:41-57, grasp.py:54-70). For env e (global id
 * g = env_offset + e), with D = num_joint_dof and W draws per env, the k-th
 * draw is the counter RNG at (seed, g * W + k):
 *   default kinds (W = 2D, s = noise_scale):
 *     qpos = default_angle + U[-s, s) (k = dof), qvel = U[-s, s) (k = D + dof)
 *   REACHER, REACHERANGLE (W = 2D + 2): the same with U[-.1, .1) and
 *     U[-.005, .005); the target (coef[0]) at (d cos a, d sin a, .01) with
 *     d = .2 u (ReacherAngle .2 sqrt(u)) at k = 2D, a = 2 pi u at k = 2D + 1
 *   PUSHER (W = D - 2): default angles, qvel U[-.005, .005) on the first
 *     D - 4 dofs (k = dof); the object (coef[1]) at U[-.3, 0) x U[-.2, .2)
 *     (k = D - 4, D - 3) scaled into a .17 disc, z = .05; the goal (coef[2])
 *     at (.45, .05, .05); the table (coef[3]) at the origin
 *   UR5E, FETCH (W = 2): the default pose at rest; the target (coef[1]) at
 *     radius coef[2] + coef[3] u (k = 0), angle 2 pi u (k = 1), z = coef[4]
 *   GRASP: the default pose at rest
 *   qp   = System.default_qp(qpos, qvel) (system.py:112-242), then the
 *          placed bodies' positions
 *   obs  = _get_obs(qp, System.info(qp), 0)    (system.py:327-340)
 *   reward = done = metrics = 0; steps = truncation = 0 when given;
 *   UR5E, FETCH, GRASP: out->rng (required) = the env's stream, a hash of
 *   (seed, g).
 * noise_scale is read by the default kinds only (the others' ranges are
 * fixed by the reference envs). Keying by global env id makes the states
 * independent of how a batch is sharded over GPUs. env_seeds
 * (device, n_envs uint64, may be NULL) gives every env its own key instead,
 * as `VmapWrapper.reset` over a (B, 2) key batch (wrappers.py:79-80): env e
 * then draws from (env_seeds[e], k) and hashes (env_seeds[e], 0) for its
 * stream. The JAX threefry stream itself is parity-unpinned.
 * The params' first_qp / first_obs are not read. */
int bx_env_reset(bx_system* sys, const bx_env_params* env, int64_t n_envs, uint64_t seed,
                 int64_t env_offset, const uint64_t* env_seeds, float noise_scale,
                 const bx_env_state* out, void* stream);

/* Env observation of a state (Env._get_obs with the reset-time Info). */
int bx_env_observe(bx_system* sys, const bx_env_params* env, int64_t n_envs,
                   const bx_qp* qp, const float* act, int64_t act_stride,
                   int64_t act_width, float* obs, void* stream);

/* Joint angles and angular velocities of every joint dof (Joint.angle_vel,
 * joints.py:197-226,311-319,388-415; Spherical: line-of-nodes x-y'-z''
 * angles), in joint order: angle and vel are (B, num_joint_dof) contiguous
 * (num_joint_dof counted after sphericalisation). */
int bx_system_joint_angles(bx_system* sys, int64_t n_envs, const bx_qp* qp, float* angle,
                           float* vel, void* stream);

/* Counter-based uniform [lo,hi) fill: out[i] = U(seed, offset + i), a
 * splitmix64 hash of (seed, global index); the same stream bx_env_reset draws
 * its noise from. Used for synthetic actions (offset = global env id x width,
 * so shards reproduce one big batch) and reset noise (the JAX threefry stream
 * is parity unpinned). */
int bx_uniform(float* out, int64_t n, uint64_t seed, uint64_t offset,
               float lo, float hi, void* stream);

/* bx_uniform with the offset read on the device: out[i] = U(seed, offset +
 * (*epoch) * epoch_stride + i), `epoch` a device int64 the caller advances
 * in stream order. A hipGraph-captured rollout (brax_amd.envs.graph) replays
 * the same launch and still draws a fresh slab per replay, exactly the slab
 * bx_uniform would draw at offset + epoch * epoch_stride (ABI 8). */
int bx_uniform_epoch(float* out, int64_t n, uint64_t seed, uint64_t offset,
                     const int64_t* epoch, uint64_t epoch_stride,
                     float lo, float hi, void* stream);

/* n_slabs slabs of slab_n elements in one launch, each slab at its own
 * offset: out[s * slab_n + j] = U(seed, offset + (*epoch) * epoch_stride +
 * s * slab_stride + j), epoch NULL reading as 0. A graph-captured rollout of K
 * steps draws its K action slabs with one launch (slab_stride = the job's
 * per-step stride world x B x A, so every slab is bit-identical to the
 * bx_uniform draw of that step; ABI 9). The bx_uniform* calls launch on the
 * device that owns `stream` (the current device for NULL). */
int bx_uniform_slabs(float* out, int64_t slab_n, int64_t n_slabs, uint64_t seed,
                     uint64_t offset, uint64_t slab_stride, const int64_t* epoch,
                     uint64_t epoch_stride, float lo, float hi, void* stream);

/*
 * Standalone HBM-streaming phase kernels over a structure-of-arrays batch
 * (the integrator and collider phases benchmarked in isolation).
 * SoA: field plane k, body b, env e at base[k*plane + b*n_envs + e]; the 13
 * state planes are pos xyz, rot wxyz, vel xyz, ang xyz. n_envs % 4 == 0,
 * planes 16-byte aligned.
 *   which 0: Euler.kinetic              (integrators.py:50-68)   in -> out pos, rot
 *   which 1: Euler.update(acc_p=aux)    (integrators.py:85-93)   aux = dp vel 3 + ang 3 planes
 *   which 2: Euler.velocity_projection  (integrators.py:122-146) aux = previous state planes
 */
int bx_phase(bx_system* sys, int which, int64_t n_envs, int64_t plane, const float* in,
             float* out, const float* aux, int64_t aux_plane, void* stream);

/* capsule_plane contacts (colliders.py:744-759) of every capsule-plane row:
 * out planes pos xyz, vel xyz, normal xyz, penetration, each (R, n_envs). */
int bx_phase_capsule_plane(bx_system* sys, int64_t n_envs, int64_t plane, const float* in,
                           float* out, int64_t out_plane, void* stream);

/* Diagnostic builds only (-DBX_STAMPS): per-phase s_memtime cycle sums of the
 * single-mode step, [0..9] phases, [15] samples; with reset bit 1 set, the
 * MULTI-mode step's (-DBX_MSTAMPS), [0..10]; with bit 2 set (single-mode),
 * the per-workgroup sums, 4096 x 16 entries. Fails on product builds. */
int bx_debug_stamps(unsigned long long* out16, int reset);

/* The revolute joint halves' partner exchange on its own (diagnostic): one
 * wavefront writes out64[l] = the value lane l receives from its partner lane
 * (l ^ 8 within each env of `lanes` = 16 threads) when every lane offers its
 * own index. */
int bx_debug_partner(float* out64, int lanes, void* stream);

/* Multi-rank episodic exchange is done over RCCL by the host (torch.distributed);
 * no collective lives in this library. */

#ifdef __cplusplus
}
#endif
#endif /* BRAX_AMD_H_ */
