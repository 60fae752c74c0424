/*
 * usv_hip.h — C-ABI of libusvhip.so, the MI355X-native batched USV path-following
 * environment (usv-simple / usv-asmc-simple step on gfx950).
 *
 * Drop-in boundary.  The reference (romi2002/gym-usv) is pure Python; its interface for
 * this path is the Gymnasium Env API of its env classes, driven N-at-a-time by SB3's
 * DummyVecEnv (train_test/sb3_train_vec.py:67).  Each entry point below replaces:
 *
 *   usv_create      <- gymnasium.make(env_id) x N / UsvSimpleEnv.__init__
 *                      (gym_usv/__init__.py:24-34, gym_usv/envs/simple_env.py:10-60,
 *                       gym_usv/envs/simple_env_asmc.py:10-12)
 *   usv_seed        <- Env.reset(seed=...) seeding of np_random (simple_env.py:229)
 *   usv_reset       <- UsvSimpleEnv.reset (simple_env.py:228-308),
 *                      UsvSimpleASMCEnv.reset (simple_env_asmc.py:14-16),
 *                      UsvAsmcEnv.reset (usv_asmc_env.py:258-300),
 *                      UsvAsmcYeIntEnv.reset (usv_asmc_ye_int_env.py:256-296),
 *                      UsvPidEnv.reset (usv_pid_env.py:236-276)
 *   usv_reset_ex    <- UsvSimpleEnv.reset(options={'place_obstacles_on_path': k}) (:276-288) and
 *                      its info dict _get_info(-1, zeros(3)) (simple_env.py:102-115, :305)
 *   usv_set_experiment <- UsvSimpleEnv(options={'run_custom_experiment': ..}) (:10, :292-300)
 *   usv_step_ex     <- the step's info dict (simple_env.py:102-115, 189-199, 343-344)
 *   usv_step        <- UsvSimpleEnv.step (simple_env.py:310-346),
 *                      UsvSimpleASMCEnv.step (simple_env_asmc.py:18-27) -> UsvAsmc.compute
 *                      (gym_usv/control/usv_asmc.py:53-244), lidar
 *                      (gym_usv/envs/usv_asmc_ca_env.py:411-461,500-519), TimeLimit
 *                      (gym_usv/__init__.py:27,33) and DummyVecEnv same-step autoreset;
 *                      legacy UsvAsmcEnv.step (usv_asmc_env.py:99-255, compute_reward :364-374),
 *                      UsvAsmcYeIntEnv.step (usv_asmc_ye_int_env.py:92-253, :350-360),
 *                      UsvPidEnv.step (usv_pid_env.py:89-233, :329-338)
 *   usv_asmc_compute <- UsvAsmc.compute (gym_usv/control/usv_asmc.py:53-244), the controller
 *                      on its own, as the reference's tests drive it (tests/test_usv_asmc.py:8-37)
 *   usv_get_field / usv_set_field / usv_get_state / usv_set_state
 *                   <- the env attributes (position, velocity, obstacle_positions, ...);
 *                      used for checkpointing and for parity state injection
 *
 * Conventions: plain pointers and sizes, no torch / HIP types.  `stream` is a hipStream_t
 * passed as void* (NULL = default stream).  Device pointers (`*_dev`) are caller-owned
 * device memory (e.g. torch tensors' data_ptr()).  Launches are asynchronous and
 * stream-ordered.  Every function returns 0 on success or a negative usv_status; the
 * message is in usv_last_error() (thread-local).  A handle is not thread-safe; use one
 * handle per device (one process per GPU).
 */
#ifndef USV_HIP_H
#define USV_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define USV_ABI_VERSION 5
#define USV_SENSOR_COUNT 128
#define USV_OBS_DIM 143      /* 15 + 128, simple_env.py:27 */
#define USV_ACT_DIM 2        /* simple_env.py:30 */
#define USV_ASMC_STATE 16    /* unique UsvAsmc state values (usv_asmc.py:43-49) */

typedef enum usv_status {
  USV_OK = 0,
  USV_ERR_ARG = -1,
  USV_ERR_HIP = -2,
  USV_ERR_ABI = -3,
  USV_ERR_STATE = -4
} usv_status;

typedef enum usv_mode {
  USV_MODE_SIMPLE = 0,       /* id "usv-simple"      (UsvSimpleEnv)                      */
  USV_MODE_ASMC_SIMPLE = 1,  /* id "usv-asmc-simple" (UsvSimpleASMCEnv)                  */
  USV_MODE_ASMC_V0 = 2,      /* id "usv-asmc-v0" legacy UsvAsmcEnv (usv_asmc_env.py:14): */
                             /* obs 6, scalar action, no lidar, no TimeLimit             */
  USV_MODE_ASMC_YE_INT_V0 = 3, /* id "usv-asmc-ye-int-v0" UsvAsmcYeIntEnv               */
                               /* (usv_asmc_ye_int_env.py:14): float64, ye integral      */
  USV_MODE_PID_V0 = 4          /* id "usv-pid-v0" UsvPidEnv (usv_pid_env.py:14): float64 */
} usv_mode;

typedef enum usv_precision { USV_F32 = 0, USV_F64 = 1 } usv_precision;

typedef enum usv_autoreset {
  USV_AUTORESET_SAME_STEP = 0, /* done envs reset inside usv_step (SB3 DummyVecEnv) */
  USV_AUTORESET_DISABLED = 1   /* done envs keep stepping until usv_reset(mask)       */
} usv_autoreset;

typedef enum usv_reset_rng {
  USV_RESET_PHILOX = 0,      /* Philox4x32-10 keyed by (seed, global env id, episode): the
                                reference's reset distributions, not its streams (default)   */
  USV_RESET_NUMPY_PCG64 = 1  /* each env's own numpy Generator(PCG64) (USV_FIELD_NP_RNG), drawn
                                in the reference's order: resets equal the reference's; the
                                legacy *-v0 ids draw from np.random's MT19937 (USV_FIELD_NP_MT) */
} usv_reset_rng;

typedef enum usv_lidar_algo {
  USV_LIDAR_BRUTE = 0,  /* every (ray, obstacle) pair                         */
  USV_LIDAR_WINDOW = 1  /* angular-window pruning, bit-identical to BRUTE    */
} usv_lidar_algo;

typedef struct usv_config {
  int32_t abi_version;       /* must be USV_ABI_VERSION */
  int32_t mode;              /* usv_mode */
  int32_t precision;         /* usv_precision: state + arithmetic type; obs is always f32 */
  int32_t num_envs;          /* envs owned by this handle */
  int32_t obstacle_cap;      /* max obstacles per env (reference draws 15..29) */
  int32_t max_episode_steps; /* TimeLimit; 0 = none. 500 usv-simple, 1000 usv-asmc-simple */
  int32_t autoreset;         /* usv_autoreset */
  int32_t lidar_algo;        /* usv_lidar_algo */
  uint64_t seed;             /* Philox key for in-kernel resets */
  uint64_t env_id_offset;    /* global id of env 0 (sharding across GPUs) */
  int32_t flags;             /* usv_flags */
  int32_t reserved;          /* 0 */
} usv_config;

typedef enum usv_flags {
  /* usv-asmc-simple: UsvAsmc.compute(..., do_perturb=True) (gym_usv/control/usv_asmc.py:184-199):
     a sinusoidal force is added to the thrust every substep; the controller's perturb_step is
     20 * elapsed + substep (a fresh UsvAsmc per episode, 2 x 10 substeps per env step) */
  USV_FLAG_PERTURB = 1
} usv_flags;

/* Per-step info (opt-in, usv_step_ex / usv_reset_ex): one row of USV_INFO_DIM values per env, in the
 * handle's precision (f32, or f64 for USV_F64: usv_reward_bytes gives the element size),
 * the keys of UsvSimpleEnv._get_info + reward_info (gym_usv/envs/simple_env.py:102-115,189-199).
 * "reward" is rew_dev itself; keys that are constant in the reference (left/right_thruster = 0,
 * angle_action_reward = 0) are not stored.  After an explicit reset the row is
 * _get_info(-1, zeros(3)) (:305): the reward-term entries are 0.  With same-step autoreset the
 * row of a done env keeps its terminal step's info. */
typedef enum usv_info_key {
  USV_INFO_X = 0, USV_INFO_Y, USV_INFO_PSI,      /* 'position' (after the step)            */
  USV_INFO_U, USV_INFO_V, USV_INFO_R,            /* 'velocity'                             */
  USV_INFO_PATH_X0, USV_INFO_PATH_Y0,            /* 'path_start'                           */
  USV_INFO_PATH_X1, USV_INFO_PATH_Y1,            /* 'path_end'                             */
  USV_INFO_ACTION0, USV_INFO_ACTION1,            /* 'action0', 'action1' (filtered action)  */
  USV_INFO_YE,                                   /* 'ye'                                   */
  USV_INFO_ANGLE_TO_TARGET,                      /* 'angle_to_target' (= angle / pi)       */
  USV_INFO_YE_REWARD, USV_INFO_ANGLE_TO_TARGET_REWARD, USV_INFO_DELTA_ACTION_REWARD,
  USV_INFO_DELTA_ACTION, USV_INFO_VELOCITY_TRACK_REWARD,
  USV_INFO_REFERENCE_VELOCITY, USV_INFO_REWARD_VELOCITY, USV_INFO_REFERENCE_VELOCITY_ERROR,
  USV_INFO_DIM
} usv_info_key;

/* reset(options=...) of UsvSimpleEnv.reset (simple_env.py:276-288) */
typedef struct usv_reset_options {
  int32_t place_obstacles_on_path;  /* k > 0: k extra obstacles scattered along the path;
                                       needs obstacle_cap >= 29 + k */
  int32_t reserved;
} usv_reset_options;

/* __init__(options={'run_custom_experiment': True, 'experiment': {...}}) of UsvSimpleEnv
 * (simple_env.py:10,292-300): every reset (explicit or autoreset) of every env of the handle
 * replaces the drawn obstacles, path and pose by these, after the usual draws. */
typedef struct usv_experiment {
  int32_t n_obs;               /* 1 .. obstacle_cap */
  int32_t reserved;
  double obstacle_x[64], obstacle_y[64], obstacle_r[64];  /* 'obstacle_positions', 'obstacle_radius' */
  double path_start[2];        /* 'path_start' */
  double angle;                /* 'angle': path_end = path_start + (cos, sin)(angle) * 100 */
  double position[3];          /* 'position' (x, y, psi) */
} usv_experiment;

/* Per-env state fields.  Host-side layout for get/set: [num_envs][per_env] row-major,
 * float64 for real fields, int32 for integer fields (usv_field_info tells which). */
typedef enum usv_field {
  USV_FIELD_X = 0, USV_FIELD_Y, USV_FIELD_PSI,          /* position (simple_env.py:39) */
  USV_FIELD_U, USV_FIELD_V, USV_FIELD_R,                /* velocity (:38)              */
  USV_FIELD_LAST_U, USV_FIELD_LAST_R,                   /* last_action[0], [2] (:41)   */
  USV_FIELD_PROGRESS,                                   /* progress (:53)              */
  USV_FIELD_PATH_X0, USV_FIELD_PATH_Y0,                 /* path_start (:51)            */
  USV_FIELD_PATH_X1, USV_FIELD_PATH_Y1,                 /* path_end (:52)              */
  USV_FIELD_MAX_U, USV_FIELD_MAX_R,                     /* max_action[0], [2] (:32)    */
  USV_FIELD_REF_V,                                      /* reference_velocity (:33)    */
  USV_FIELD_N_OBS,          /* int: obstacle_n (:44)                                    */
  USV_FIELD_ELAPSED,        /* int: TimeLimit elapsed steps                              */
  USV_FIELD_EPISODE,        /* int: episode counter (Philox counter word)                */
  USV_FIELD_SCAN_VALID,     /* int: 1 if the current pose's scan is the stale sensor_data */
  USV_FIELD_OBS_X, USV_FIELD_OBS_Y, USV_FIELD_OBS_R,    /* [cap] obstacles (:45-46)    */
  USV_FIELD_SENSOR_LAST,    /* [128] stale scan for reset obs (sensor_data, :47)          */
  USV_FIELD_ASMC,           /* [16] UsvAsmc state (usv-asmc-simple only)                  */
  USV_FIELD_V0_LAST,        /* [9]  usv-asmc-v0 `last` (eta_dot, upsilon_dot, e_u_last, Ka_dots) */
  USV_FIELD_V0_AUX,         /* [3]  usv-asmc-v0 `aux_vars` (e_u_int, Ka_u, Ka_psi)        */
  USV_FIELD_V0_TARGET,      /* [6]  usv-asmc-v0 `target` (x_0, y_0, speed, ak, x_d, y_d)  */
  USV_FIELD_V0_ACTION_LAST, /* [1]  usv-asmc-v0 state[5] (previous action)                 */
  USV_FIELD_V0_YE,          /* [2]  usv-asmc-ye-int-v0 aux_vars[3] ye_int, last[9] ye_last  */
  USV_FIELD_NP_RNG,         /* int [10]: the env's numpy Generator(PCG64) for USV_RESET_NUMPY_PCG64:
                               state high / low and increment high / low 64-bit words as
                               little-endian 32-bit halves, has_uint32, uinteger
                               (bit_generator.state of np.random.PCG64)                    */
  USV_FIELD_NP_MT,          /* int [625] (legacy *-v0 ids; 0 otherwise): np.random's global
                               RandomState MT19937 key[624] and pos, for USV_RESET_NUMPY_PCG64 */
  USV_FIELD_COUNT
} usv_field;

int usv_abi_version(void);
const char* usv_last_error(void);
/* sizeof(usv_config) as compiled into the library (56): a binding checks its own struct against it
 * (ABI v5). */
size_t usv_config_size(void);

/* Fill `cfg` with the reference defaults for `mode` (cap 32, TimeLimit by id -- 500, 1000,
 * none for the legacy *-v0 ids --, f32, same-step autoreset, window lidar, seed 0). */
void usv_config_default(usv_config* cfg, int32_t mode, int32_t num_envs);

int usv_create(const usv_config* cfg, int32_t device, void** handle_out);
void usv_destroy(void* handle);

int usv_num_envs(void* handle);
int usv_obs_dim(void* handle);   /* 143 (usv-simple, usv-asmc-simple) or 6 (legacy *-v0 ids) */
int usv_act_dim(void* handle);   /* 2, or 1 for the legacy *-v0 ids */
/* Bytes of one reward element (4 for USV_F32, 8 for USV_F64). */
int usv_reward_bytes(void* handle);

/* Re-key the reset RNG (Philox4x32-10, key = seed, counter = global env id / episode)
 * and zero every episode counter.  Host-side only; no launch. */
int usv_seed(void* handle, uint64_t seed);

/* Select the reset RNG (usv_reset_rng) <- Env.reset(seed) seeding np_random
 * (simple_env.py:229, gymnasium seeding.np_random) and np.random.seed + np.random.uniform
 * (usv_asmc_env.py:258-279).  The generator states are set through USV_FIELD_NP_RNG /
 * USV_FIELD_NP_MT. */
int usv_set_reset_rng(void* handle, int32_t kind);

/* Reset envs whose mask byte is non-zero (all envs if mask_dev == NULL) and write their
 * reset observation rows into obs_dev [num_envs][obs_dim] (other rows untouched). */
int usv_reset(void* handle, const uint8_t* mask_dev, float* obs_dev, void* stream);
/* usv_reset with reset options (NULL = none) and an optional info buffer info_dev
 * [num_envs][USV_INFO_DIM] f32 / f64 by precision (NULL = none; rows of reset envs are written). */
int usv_reset_ex(void* handle, const uint8_t* mask_dev, float* obs_dev,
                 const usv_reset_options* options, void* info_dev, void* stream);
/* Install (experiment != NULL) or remove (NULL) the custom experiment of every env. */
int usv_set_experiment(void* handle, const usv_experiment* experiment);

/* One env step for every env.
 *   act_dev       [num_envs][act_dim] f32 (u in [0.2,1], r in [-1,1]; usv-asmc-simple: (u_d, psi
 *                 offset); legacy *-v0 ids: heading offset in [-pi/2, pi/2])
 *   obs_dev       [num_envs][obs_dim] f32  (reset obs for envs that autoreset)
 *   rew_dev       [num_envs] f32 or f64 (usv_reward_bytes)
 *   term_dev, trunc_dev [num_envs] u8
 *   final_obs_dev [num_envs][obs_dim] f32 or NULL: terminal obs rows of done envs
 *                 (rows of envs not done are left untouched). */
int usv_step(void* handle, const float* act_dev, float* obs_dev, void* rew_dev,
             uint8_t* term_dev, uint8_t* trunc_dev, float* final_obs_dev, void* stream);
/* usv_step with two optional outputs (NULL = not written):
 *   done_dev  [num_envs] u8: terminated | truncated, i.e. gymnasium's info['_final_obs'] mask (ABI v4)
 *   info_dev  [num_envs][USV_INFO_DIM] f32 / f64 by precision: the per-step info rows (usv-simple /
 *             usv-asmc-simple; the legacy *-v0 ids return {} in the reference and ignore it). */
int usv_step_ex(void* handle, const float* act_dev, float* obs_dev, void* rew_dev,
                uint8_t* term_dev, uint8_t* trunc_dev, uint8_t* done_dev, float* final_obs_dev,
                void* info_dev, void* stream);

/* UsvAsmc.compute(action, position, velocity, do_perturb) (gym_usv/control/usv_asmc.py:53-244) for
 * n independent controllers, `calls` compute() calls back to back (10 substeps of 0.01 s each), in
 * place on device buffers of the precision's type (float for USV_F32, double for USV_F64):
 *   act_dev [n][2] (u_d, heading offset), pos_dev [n][3] (x, y, psi), vel_dev [n][3] (u, v, r),
 *   state_dev [16][n]: psi_d_last, o, o', o'', eta_dot_last[3], upsilon_dot_last[3], e_u_last,
 *     Ka_dot_u_last, Ka_dot_psi_last, e_u_int, Ka_u, Ka_psi (so_filter / last / aux_vars, :43-49;
 *     the reference keeps so_filter's o_last, o_dot_last, o_dot_dot_last equal to o, o', o'');
 *   perturb_step_dev int32 [n] or NULL (= 0): the controllers' perturb_step (:49), advanced by 10
 *     per call; do_perturb adds the sinusoidal disturbance (:184-199).
 * Stream-ordered, no handle (ABI v5); launched on the device that holds state_dev, whatever device is
 * current (USV_ERR_ARG if any buffer is not device memory of the device that holds state_dev). */
int usv_asmc_compute(int32_t precision, int32_t n, const void* act_dev, void* pos_dev, void* vel_dev,
                     void* state_dev, int32_t* perturb_step_dev, int32_t do_perturb, int32_t calls,
                     void* stream);

/* Select the step-kernel variant of a usv-simple / usv-asmc-simple handle (verification and
 * tuning: every variant computes bit-identical outputs, tests/test_gpu_*.py compare them bitwise).
 * No reference counterpart; usv_create picks the tuned default.
 *   kind 1: fused wave kernel (epb 16 | 32 | 64 envs per 256-thread block)
 *   kind 2: split dynamics + wave scan (epb 8 | 16 | 32; f64 usv-simple window also 64)
 *   kind 3: one launch, wave 0 of each 4-wave block runs the block's dynamics, then the wave scan
 *           (f64 usv-simple, window lidar; epb 32 | 64)
 *   kind 4 / 5: split / fused block-queue step (epb 128; kind 5 also 16), f32 window lidar, cap <= 32
 *   kind 6: usv-asmc-simple only: the ASMC chain in its own launch, then the fused block-queue step
 *           (epb 128 | 16), f32 window lidar, cap <= 32
 *   lid: lidar variant bits (0 brute, 3 brute + blind-sector skip + unroll, 7 angular window); kinds 4-6
 *        also take 0x100 / 0x200: obs rows stored as 32-B-aligned env-pair spans forced on / off (default:
 *        on from 196 608 envs, where the rows go to DRAM)
 * Waits for in-flight launches first.  USV_ERR_ARG if the handle's config cannot run it. */
int usv_set_kernel_variant(void* handle, int32_t kind, int32_t epb, int32_t lid);

/* Field metadata: values per env, 1 if int32, name. */
int usv_field_info(void* handle, int32_t field, int32_t* per_env, int32_t* is_int,
                   const char** name);
/* Synchronous host copies (device synchronised first). `bytes` must equal
 * num_envs * per_env * (is_int ? 4 : 8). */
int usv_get_field(void* handle, int32_t field, void* host, size_t bytes);
int usv_set_field(void* handle, int32_t field, const void* host, size_t bytes);

/* Whole-state blob (all fields in enum order, host layout as above): env checkpoint. */
size_t usv_state_bytes(void* handle);
int usv_get_state(void* handle, void* host, size_t bytes);
int usv_set_state(void* handle, const void* host, size_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* USV_HIP_H */
