// usv_kernels.hip — gfx950 kernels + C-ABI (include/usv_hip.h) for the batched USV
// path-following environment (usv-simple / usv-asmc-simple).
//
// One step = ONE launch over all envs.  A 256-thread block owns EPB consecutive envs:
//   phase 1  lane-per-env  (wave 0): [ASMC 2x10 substeps] + kinematics + closest point +
//            cross-track error + target features + reward terms + truncation; SoA state
//            loads/stores are coalesced [field][N]; results for phase 2 go to LDS.
//   phase 2  wave-per-env  (all 4 waves): obstacle keys (lane j = obstacle j), termination,
//            128-ray lidar (lane l = rays l, l+64; obstacle data broadcast by v_readlane so
//            the ray loop is wave-uniform), min sensor, and the whole 572-B observation row
//            written by contiguous lanes (coalesced).
//   phase 3  lane-per-env  (wave 0): reward, flags, and in-kernel masked autoreset
//            (Philox, no host round trip) for done envs.
// Reference: see include/usv_hip.h for the file:line each entry point replaces.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <type_traits>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "usv_device.hpp"
#include "usv_hip.h"

namespace usv {

// (x, y, r, r*r) of one obstacle as a native 4-vector (one 16-B / 32-B access, selectable in
// registers without a stack temporary)
template <typename R> struct V4;
template <> struct V4<float> { typedef float T __attribute__((ext_vector_type(4))); };
template <> struct V4<double> { typedef double T __attribute__((ext_vector_type(4))); };
template <typename R> using R4 = typename V4<R>::T;

enum RealField {
  F_X, F_Y, F_PSI, F_U, F_V, F_R, F_LAST_U, F_LAST_R, F_PROGRESS,
  F_PX0, F_PY0, F_PX1, F_PY1, F_MAX_U, F_MAX_R, F_REF_V, F_NREAL
};

// Device state.  All real SoA fields share one allocation (field i at freal + i*fstride) and
// the int fields another, so the kernel holds two base pointers instead of twenty (kernel
// arguments live in SGPRs; fewer of them keeps the kernel at <= 80 SGPRs = 8 blocks per CU).
// I_TURNS (f32 usv-simple / usv-asmc-simple): whole turns of the heading, see store_heading
enum IntField { I_NOBS, I_ELAPSED, I_EPISODE, I_SCAN, I_TURNS, I_NINT };
template <typename R> struct State {
  R* freal;                // [F_NREAL][fstride]
  int32_t* fint;           // [I_NINT][fstride]
  R* obst;                 // [N][3][ostride]: per env the planes x[ostride], y[ostride], r[ostride]
                           //   (slots >= n_obs zero); one env's row is 3 * ostride * sizeof(R) bytes
  R* sensor_last;          // [N][128]
  R* asmc;                 // [16][N]
  R* v0;                   // [21][fstride] legacy envs: last[9], aux[3], target[6], action_last,
                           //   ye_int, ye_last (usv-asmc-ye-int-v0)
  const R* ray_tab;        // [128][2] (cos, sin)(start + i*res)
  R4<R>* pose;             // [N][2] pose record after the step's dynamics (split wave step):
                           //   (x, y, sin psi, cos psi), (partial reward, n_obs, truncated, 0)
  float* qrec;             // [N][kQRec] f32 env record of the split block-queue step (dyn_rec_kernel)
  uint32_t* nprng;         // [10][fstride] NumPy PCG64 per env (state hi/lo, inc hi/lo as 32-bit
                           //   words, has_uint32, uinteger) for the NumPy-exact reset
  uint32_t* npmt;          // [625][fstride] legacy envs: np.random.RandomState MT19937 key[624], pos
  int np_reset;            // 1: resets draw from NumPy's Generator(PCG64) (np_reset) -- legacy
                           //   envs: from np.random's MT19937 (NpMt) -- not Philox
  int perturb;             // usv-asmc-simple: do_perturb (USV_FLAG_PERTURB)
  const R* exp;            // custom experiment applied by every reset, or null (kExp* layout)
  int N, cap, limit, autoreset;
  int prio;                // scan loops: raise the issue priority of lagging waves (s_setprio)
  int rowspan;             // block-queue step: store an env pair's obs rows as one 32-B-aligned span
  int qyoung;              // block-queue step: blocks from this index raise kQYoungWaves waves' issue
                           //   priority (a CU's second block of a one-round grid; INT_MAX: none)
  int fstride;             // elements between fields (>= N, 256-B aligned)
  int ostride;             // obstacle plane stride: cap rounded up to a multiple of 4
  uint64_t seed, gid0;
  __host__ __device__ R* F(int i) const { return freal + (size_t)i * fstride; }
  __host__ __device__ int32_t* I(int i) const { return fint + (size_t)i * fstride; }
  __host__ __device__ R* V(int i) const { return v0 + (size_t)i * fstride; }
  __host__ __device__ R* orow(int e) const { return obst + (size_t)e * 3 * ostride; }
};
constexpr int kV0Last = 0, kV0Aux = 9, kV0Target = 12, kV0ALast = 18, kV0Ye = 19, kV0N = 21;

// Heading representation of the f32 usv-simple / usv-asmc-simple state.  The reference integrates the
// heading without wrapping (simple_env.py:323, usv_asmc.py:234), so it grows without bound, and a float
// of 400 rad holds it to only +-1.5e-5 rad: every step's rounding then moved the angle feature
// (obs[3] = angle / pi) by ~5e-6 and the pose by the heading error times the distance run.  The f32
// state keeps psi = phi + 2 pi k instead: phi (F_PSI, a float within about a turn of zero) and the
// whole turns k (I_TURNS, int), with UsvAsmc's psi_d_last in phi's frame; the host state interface
// returns phi + 2 pi k in float64.  Every use of the heading is through sin / cos, wrap(. - psi) or
// differences, which are 2 pi-periodic or frame-free.  The f64 build keeps the reference's absolute
// heading (k = 0 always) and its arithmetic order.
constexpr float kTwoPiHi = 6.28318548f, kTwoPiLo = 1.74845553e-07f;   // 2 pi = hi - lo (float split)
template <typename R> __device__ __forceinline__ R turns_of(R psi) { return rint(psi * R(0.15915494309189535)); }
// psi - 2 pi n in float, the high part exact by Sterbenz for |n| <= 1 and |psi| within a turn or two
__device__ __forceinline__ float sub_turns(float psi, float n) { return fmaf(n, kTwoPiLo, fmaf(-n, kTwoPiHi, psi)); }
// A reset's heading (drawn, or the custom experiment's), with its whole turns split off in the f32 build
template <typename R> __device__ __forceinline__ void store_heading(const State<R>& S, int e, R psi) {
  if constexpr (std::is_same<R, float>::value) {
    const float n = turns_of(psi);
    S.F(F_PSI)[e] = sub_turns(psi, n);
    S.I(I_TURNS)[e] = (int)n;
  } else {
    S.F(F_PSI)[e] = psi;
  }
}
// End of an f32 step (env_dynamics): once the heading phi has left [-pi, pi], its whole turns move
// into k, and (usv-asmc-simple) UsvAsmc's psi_d_last with it, so the stored phi is always within
// [-pi, pi] and the host's phi + 2 pi k splits back into the same (phi, k).  k and psi_d_last are
// loaded with the rest of the state and stored back plain: a load after the dynamics' stores would
// make the wave wait for their acks (one vmcnt counter), and atomic adds are wrong for the lanes that
// repeat a wave's last env (each would add the turns again), where plain stores of the same value
// are not.
// phi + 2 pi k (the reference's heading) in R: for the info row
template <typename R> __device__ __forceinline__ R heading_abs(R phi, int k) {
  if constexpr (std::is_same<R, float>::value) {
    const float kf = (float)k;
    return fmaf(-kf, kTwoPiLo, fmaf(kf, kTwoPiHi, phi));
  } else {
    return phi;
  }
}
// custom experiment record (usv_experiment, simple_env.py:292-300), in R: n, path start (2),
// path angle, pose (3), pad, then x[cap], y[cap], r[cap]
constexpr int kExpN = 0, kExpPS = 1, kExpAngle = 3, kExpPose = 4, kExpObs = 8;

template <typename R> struct IO {
  const float* act;        // [N][2]
  float* obs;              // [N][143]
  R* rew;                  // [N]
  uint8_t* term;           // [N]
  uint8_t* trunc;          // [N]
  float* fobs;             // [N][143] or null
  const uint8_t* mask;     // [N] or null (reset kernel)
  R* info;                 // [N][USV_INFO_DIM] in R (f32 / f64 build) or null: step info (step kernels) / reset info
  int kpath;               // reset kernel: options['place_obstacles_on_path'] (0 = none)
  uint8_t* done;           // [N] terminated | truncated (gymnasium's info['_final_obs']) or null
};

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / kWave;
constexpr int kEPBReset = 64;   // envs per block of the reset kernel
constexpr int kLidDefault = 7;  // lidar variant of the reset kernel (all variants give identical scans)

template <typename R> __device__ __forceinline__ R big() { return R(1e30); }

#ifdef USV_DIAG
#include "usv_diag.hpp"       // diagnostic builds only: per-block / per-wave clock stamps
#else
#define USV_STAMP_ID() do {} while (0)
#define USV_STAMP(i) do {} while (0)
#define USV_STAMP_B(i) do {} while (0)
#define USV_STAMP_W(i) do {} while (0)
#define USV_STAMP_V(i, v) do {} while (0)
struct Prof {
  __device__ void mark(int) {}
  __device__ void count(int) {}
  __device__ void flush(int) {}
};
struct QProf { __device__ void mark(int) {} __device__ void count(int, unsigned = 1) {} __device__ void flush() {} };
#define QMARK(i) do {} while (0)
#define QCOUNT(i, k) do {} while (0)
__device__ __forceinline__ void qprof_flush(QProf*) {}
#endif
// Output rows (obs, reward) are stored write-through (sc1: the line leaves the XCD's L2 as it is
// written, instead of being written back at the kernel boundary) where a wave stores contiguous
// bytes (a row's sensors, consecutive envs' rewards); lane-per-env stores to 64 different rows stay
// plain, so that L2 merges them.  The next launch on the stream
// then starts without a write-back of ~40 MB of dirty obs lines: 20.9 -> 19.4 us per step at
// 65 536 envs (back-to-back launches, tools/exp_ab.sh); the same policy for the dynamics' state
// stores measured slower (19.8 us), non-temporal stores in between (20.1 us).
template <typename T> __device__ __forceinline__ void st_out(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // global_store ... sc1
}
// obs-row stores of the block-queue step: write-through like st_out
template <typename T> __device__ __forceinline__ void st_obs(T* p, T v) { st_out(p, v); }

// Obs-row store layout of the block-queue step (State::rowspan; usv_set_kernel_variant lid bits 0x100 /
// 0x200 force it on / off; a template switch, SPAN, of the 128-env fused kernels without info rows, as
// the two layouts' code together in the pair loop spilled SGPRs; the others store pieces): an env pair's two rows as one span of 32-B-aligned 256-B stores (round 4),
// or each row in pieces (the sensor halves, then both headers in one store).  The span writes
// 1.05x the algorithmic bytes (pieces: 1.18x, sectors split between write-through stores) and wins
// where the rows go to DRAM (524 288 envs: 183.4 -> 161.4 us per step); with the working set in the
// 256 MB Infinity Cache the pieces are faster (65 536 envs: 19.2 vs 20.3 us), so the default switches
// at kRowSpanFrom envs.
constexpr int kRowSpanFrom = 196608;
// issue-priority mode of the static-split kinds 1-3 (State::prio: 1 ramp, 2 last iteration first, 0 none);
// kind 3 f64 at 65 536 envs, same box: 1 -> 40.5 us, 0 -> 43.2, 2 -> 43.2
constexpr int kStaticPrio = 1;

// Division and square root of the per-step dynamics: in the f32 build the hardware reciprocal and
// square root (1 ulp; the reference's float64 values are matched to SURVEY 8(c)'s tolerance), which
// shortens the dependent chain of the block queue's phase 1 (barrier exit 3.4 -> 2.6 us); IEEE in
// the f64 build.
template <typename R> __device__ __forceinline__ R dyn_div(R a, R b) { return a / b; }
template <typename R> __device__ __forceinline__ R dyn_sqrt(R x) { return m_sqrt(x); }
template <> __device__ __forceinline__ float dyn_div(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }
template <> __device__ __forceinline__ float dyn_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }

template <typename R> struct Vec2;
template <> struct Vec2<float> { using T = float2; };
template <> struct Vec2<double> { using T = double2; };

// obs[0:15] = [velocity/10, target_state(4), last_action[[0,2]]/max_action[[0,2]],
//              max_action/10, max_acceleration/10]   (simple_env.py:72-96)
// x / c for a compile-time constant c: correctly rounded in the f64 build (div_const), a multiply by the
// rounded reciprocal (<= 1 ulp) in the f32 build.
template <typename R> __device__ __forceinline__ R cdiv(R x, double c) { return div_const(x, c); }
template <> __device__ __forceinline__ float cdiv(float x, double c) { return x * (float)(1.0 / c); }

template <typename R>
__device__ __forceinline__ void make_header(float (&h)[kHdr], R u, R v, R r, R angle, R dist,
                                            R ye, R refv, R act_u, R act_r, R mu, R mr) {
  h[0] = (float)cdiv(u, 10); h[1] = (float)cdiv(v, 10); h[2] = (float)cdiv(r, 10);
  h[3] = (float)cdiv(angle, kPi); h[4] = (float)cdiv(dist, kDiag);
  h[5] = (float)cdiv(ye, 10); h[6] = (float)cdiv(refv, 10);
  h[7] = (float)dyn_div(act_u, mu); h[8] = (float)dyn_div(act_r, mr);
  h[9] = (float)cdiv(mu, 10); h[10] = 0.0f; h[11] = (float)cdiv(mr, 10);
  h[12] = (float)(kMaxAccU / 10.0); h[13] = 0.0f; h[14] = (float)(kMaxAccR / 10.0);
}

// --------------------------------------------------------------------------- reset
// In-kernel episode reset of env e, executed by one whole wave (wave-parallel), and
// distributionally identical to UsvSimpleEnv.reset (simple_env.py:228-308).
//
// Random numbers: lane l runs two Philox4x32-10 blocks keyed by the run seed with counter
// (global env id, episode, l) and (global env id, episode, l + 64): four 53-bit uniforms
// U[l][0..3].  Lane j < 32 draws obstacle j (x, y, radius); lanes 32..36 draw the scalars.
// The reference's draw order cannot be reproduced with Philox anyway (PCG64 + ziggurat), so
// parity of resets is distributional (KS tests); the stream is fixed per (seed, env, episode),
// independent of sharding, precision and kernel.
// last_action is NOT reset (reference quirk) and sensor_data stays stale (the caller keeps the
// scan in the obs row).  Writes the reset-obs header into row[0:15].
// Four uniforms in [0, 1) per lane: one Philox block (24-bit floats) for the f32 build, two
// blocks (53-bit doubles) for the f64 build.
template <typename R> struct Uni4 { R u[4]; };
__device__ __forceinline__ void philox_uniforms(Philox& g, int l, Uni4<float>& o) {
  uint32_t a[4];
  g.c3 = (uint32_t)l;
  g.block(a[0], a[1], a[2], a[3]);
#pragma unroll
  for (int i = 0; i < 4; ++i) o.u[i] = (float)(a[i] >> 8) * (1.0f / 16777216.0f);
}
__device__ __forceinline__ void philox_uniforms(Philox& g, int l, Uni4<double>& o) {
  uint32_t a[4], b[4];
  g.c3 = (uint32_t)l;
  g.block(a[0], a[1], a[2], a[3]);
  g.c3 = (uint32_t)l + 64u;
  g.block(b[0], b[1], b[2], b[3]);
  const double k = 1.0 / 9007199254740992.0;
  o.u[0] = (double)((((uint64_t)a[0] << 32) | a[1]) >> 11) * k;
  o.u[1] = (double)((((uint64_t)a[2] << 32) | a[3]) >> 11) * k;
  o.u[2] = (double)((((uint64_t)b[0] << 32) | b[1]) >> 11) * k;
  o.u[3] = (double)((((uint64_t)b[2] << 32) | b[3]) >> 11) * k;
}

// Reset info row _get_info(-1, zeros(3)) (simple_env.py:102-115, :305); reward terms 0.
template <typename R>
__device__ __forceinline__ void reset_info(R* info, R x, R y, R psi, R u, R v, R r, R px0, R py0,
                                           R px1, R py1, R ye, R angle_n) {
  const R vals[USV_INFO_DIM] = {x, y, psi, u, v, r, px0, py0, px1, py1, R(0), R(0),
                                ye, angle_n, R(0), R(0), R(0), R(0), R(0), R(0), R(0), R(0)};
#pragma unroll
  for (int i = 0; i < USV_INFO_DIM; ++i) info[i] = vals[i];
}

// cross-track error of (x, y) w.r.t. the path (simple_env.py:133-137); sin/cos of the path angle
// a_k = atan2(dy, dx) are dy/|d| and dx/|d|
template <typename R>
__device__ __forceinline__ R path_ye(R x, R y, R x0, R y0, R x1, R y1) {
  const R dx = x1 - x0, dy = y1 - y0;
  const R inv_len = R(1) / m_sqrt(dx * dx + dy * dy);
  return -(x - x0) * (dy * inv_len) + (y - y0) * (dx * inv_len);
}

// run_custom_experiment (simple_env.py:292-300): after the usual draws of a reset, the drawn
// obstacles, path and pose are replaced by the experiment's; target, velocity and action limits
// stay drawn.  One lane per env: it re-derives the drawn scalars of episode `ep` from their Philox
// lanes (33..35 of reset_wave), then rewrites obstacles, state, the obs header and info.  Run by
// the reset kernel after reset_wave and, for same-step autoresets, by exp_autoreset_kernel after
// the step (kept out of the step kernels, whose pair loop it would make spill).
template <typename R>
__device__ __forceinline__ void reset_experiment(const State<R>& S, int e, int ep, float* row, R* info) {
  const R* X = S.exp;
  R tx, ty, u, v, r, mu, mr, refv;
  {
    Philox g(S.seed, S.gid0 + (uint64_t)e, (uint32_t)ep);
    Uni4<R> U33, U34, U35;
    philox_uniforms(g, 33, U33);
    philox_uniforms(g, 34, U34);
    philox_uniforms(g, 35, U35);
    tx = R(kBound) * U33.u[1]; ty = R(kBound) * U33.u[2];
    u = R(0.15) * U33.u[3]; v = R(0.15) * U34.u[0]; r = R(0.15) * U34.u[1];
    mu = R(1.5) + R(1.5) * U34.u[2];
    mr = R(3) + R(3) * U34.u[3];
    refv = R(0.75) + (mu - R(0.75)) * U35.u[0];
  }
  const int cnt = (int)X[kExpN];
  R* ob = S.orow(e);
  for (int j = 0; j < S.cap; ++j) {
    ob[j] = j < cnt ? X[kExpObs + j] : R(0);
    ob[S.ostride + j] = j < cnt ? X[kExpObs + S.cap + j] : R(0);
    ob[2 * S.ostride + j] = j < cnt ? X[kExpObs + 2 * S.cap + j] : R(0);
  }
  const R ps0 = X[kExpPS], ps1 = X[kExpPS + 1];
  R sx2, cx2;
  m_sincos(X[kExpAngle], &sx2, &cx2);
  const R pe0 = ps0 + cx2 * R(100), pe1 = ps1 + sx2 * R(100);                     // :296
  const R px = X[kExpPose], py = X[kExpPose + 1], psi = X[kExpPose + 2];
  S.F(F_X)[e] = px; S.F(F_Y)[e] = py;
  store_heading<R>(S, e, psi);
  S.F(F_PX0)[e] = ps0; S.F(F_PY0)[e] = ps1;
  S.F(F_PX1)[e] = pe0; S.F(F_PY1)[e] = pe1;
  S.I(I_NOBS)[e] = cnt;
  const R angle = wrap_angle(m_atan2(ty - py, tx - px) - psi);                    // :302, :63-80
  const R dst = m_hypot(px - tx, py - ty);
  const R ye = path_ye(px, py, ps0, ps1, pe0, pe1);
  float h[kHdr];
  make_header<R>(h, u, v, r, angle, dst, ye, refv, R(0), R(0), mu, mr);
  for (int i = 0; i < kHdr; ++i) row[i] = h[i];
  if (info) reset_info<R>(info, px, py, psi, u, v, r, ps0, ps1, pe0, pe1, ye, cdiv(angle, kPi));
}

template <typename R, int MODE>
__device__ __forceinline__ void reset_wave(const State<R>& S, int e, float* row, R* info = nullptr,
                                           int kpath = 0) {
  if (S.np_reset) return;                  // NumPy-exact mode: np_autoreset_kernel resets after the step
  const int l = lane_id();
  const int ep = uniform(S.I(I_EPISODE)[e]);
  Philox g(S.seed, S.gid0 + (uint64_t)e, (uint32_t)ep);
  Uni4<R> U;
  philox_uniforms(g, l, U);
  // scalar draws (uniform across the wave, held in SGPRs):
  //   lane 32: path-start normal pair (Box-Muller) (:234-235), psi (:238), path angle (:241)
  //   lane 33: path length (:242), target x, y (:245), u0 (:246)
  //   lane 34: v0, r0 (:246), max_action[0] (:249), max_action[2] (:250)
  //   lane 35: ref_v (:251), obstacle count (:257), fallback obstacle x, y (:273)
  //   lane 36: fallback obstacle radius (:290)
  const R bm = m_sqrt(R(-2) * log(R(1) - bcast(U.u[0], 32)));
  R sb, cb;
  m_sincos(R(2 * kPi) * bcast(U.u[1], 32), &sb, &cb);
  const R sx = R(kBound / 2) + R(0.5) * bm * cb, sy = R(kBound / 2) + R(0.5) * bm * sb;
  const R tx = R(kBound) * bcast(U.u[1], 33), ty = R(kBound) * bcast(U.u[2], 33);
  const R mu = R(1.5) + R(1.5) * bcast(U.u[2], 34);
  const int n = min(15 + (int)(bcast(U.u[1], 35) * R(15)), 29);
  // obstacles: lane j < n draws (x, y) in [0, 20]^2 (:258) and its radius (:290); drop those
  // within 0.5 of the start or the target (:261-268), order kept; none left -> one fallback
  const R ox = R(kBound) * U.u[0], oy = R(kBound) * U.u[1], orad = R(0.15) + R(0.35) * U.u[2];
  const bool keep = (l < n) && !(m_hypot(sx - ox, sy - oy) < R(0.5) || m_hypot(tx - ox, ty - oy) < R(0.5));
  const unsigned long long ball = ballot(keep);
  int cnt = __popcll(ball);
  const int pos = __builtin_amdgcn_mbcnt_hi((unsigned)(ball >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)ball, 0));
  R* ob = S.orow(e);
  const int os = S.ostride;
  if (keep) { ob[pos] = ox; ob[os + pos] = oy; ob[2 * os + pos] = orad; }
  if (cnt == 0) {
    const R fx = R(kBound) * bcast(U.u[2], 35), fy = R(kBound) * bcast(U.u[3], 35);
    const R fr = R(0.15) + R(0.35) * bcast(U.u[0], 36);
    if (l == 0) { ob[0] = fx; ob[os] = fy; ob[2 * os] = fr; }
    cnt = 1;
  }
  const R ang = R(-kPi) + R(2 * kPi) * bcast(U.u[3], 32);
  if (kpath > 0) {
    // options['place_obstacles_on_path'] (:276-288): k obstacles at N(path_start + (cos, sin)(angle)
    // * U(0, hypot(0, 20) = 20), 1) per axis, appended unfiltered; lane j draws obstacle j from the
    // Philox block at counter j + 128 (explicit resets only: the step kernels pass kpath = 0)
    R sa, ca;
    m_sincos(ang, &sa, &ca);
    Uni4<R> P;
    philox_uniforms(g, l + 128, P);
    const R mag = R(kBound) * P.u[0];
    const R bq = m_sqrt(R(-2) * log(R(1) - P.u[1]));
    R s2, c2;
    m_sincos(R(2 * kPi) * P.u[2], &s2, &c2);
    const R lx = (ca * mag + sx) + bq * c2, ly = (sa * mag + sy) + bq * s2;
    const R lr = R(0.15) + R(0.35) * P.u[3];
    if (l < kpath) { ob[cnt + l] = lx; ob[os + cnt + l] = ly; ob[2 * os + cnt + l] = lr; }
    cnt += kpath;
  }
  if (l >= cnt && l < S.cap) { ob[l] = R(0); ob[os + l] = R(0); ob[2 * os + l] = R(0); }
  if (MODE == USV_MODE_ASMC_SIMPLE && l < kAsmcN) S.asmc[(size_t)l * S.N + e] = R(0);  // simple_env_asmc.py:15
  if (l == 0) {
    const R psi = R(-kPi) + R(2 * kPi) * bcast(U.u[2], 32);
    const R dist = R(100) + R(10) * bcast(U.u[0], 33);
    const R u = R(0.15) * bcast(U.u[3], 33), v = R(0.15) * bcast(U.u[0], 34), r = R(0.15) * bcast(U.u[1], 34);
    const R mr = R(3) + R(3) * bcast(U.u[3], 34);
    const R refv = R(0.75) + (mu - R(0.75)) * bcast(U.u[0], 35);
    R sa, ca;
    m_sincos(ang, &sa, &ca);
    S.F(F_X)[e] = sx; S.F(F_Y)[e] = sy;
    store_heading<R>(S, e, psi);
    S.F(F_U)[e] = u; S.F(F_V)[e] = v; S.F(F_R)[e] = r;
    S.F(F_PROGRESS)[e] = R(0);
    S.F(F_PX0)[e] = sx; S.F(F_PY0)[e] = sy;
    S.F(F_PX1)[e] = sx + ca * dist; S.F(F_PY1)[e] = sy + sa * dist;                // :243
    S.F(F_MAX_U)[e] = mu; S.F(F_MAX_R)[e] = mr; S.F(F_REF_V)[e] = refv;
    S.I(I_NOBS)[e] = cnt;
    S.I(I_ELAPSED)[e] = 0;
    S.I(I_EPISODE)[e] = ep + 1;
    S.I(I_SCAN)[e] = 0;
    // reset obs: _get_obs(zeros(3)) with the random target_position (:302, :72-80); position
    // == path_start, so ye == 0 exactly
    const R angle = wrap_angle(m_atan2(ty - sy, tx - sx) - psi);
    const R dst = m_hypot(sx - tx, sy - ty);
    float h[kHdr];
    make_header<R>(h, u, v, r, angle, dst, R(0), refv, R(0), R(0), mu, mr);
#pragma unroll
    for (int i = 0; i < kHdr; ++i) row[i] = h[i];
    if (info) reset_info<R>(info, sx, sy, psi, u, v, r, sx, sy, sx + ca * dist, sy + sa * dist, R(0), cdiv(angle, kPi));
  }
}

// sin/cos of the heading used by the lidar; the step kernel and the reset kernel (stale scan)
// must use this same function so their scans are bit-identical
template <typename R> __device__ __forceinline__ void heading_sincos(R psi, R* s, R* c) { fx_sincos(psi, s, c); }


// --------------------------------------------------------------------------- NumPy-exact reset
// numpy.random.Generator(PCG64) as the reference's reset uses it (simple_env.py:234-290), one lane
// per env, draws in the reference order: PCG64 (128-bit LCG, XSL-RR output, stepped before each
// output), next_uint32 buffering the high half, next_double = (next64 >> 11) * 2^-53, the
// ziggurat standard normal over NumPy's tables, uniform = lo + (hi - lo) * next_double and
// Lemire's 32-bit bounded integers.  oracle/np_rng.py restates it and is checked against numpy.
#include "np_ziggurat.inc"
struct NpPcg64 {
  uint64_t sh, sl, ih, il;
  uint32_t has32, u32;
  __device__ uint64_t next64() {
    constexpr uint64_t kMh = 2549297995355413924ULL, kMl = 4865540595714422341ULL;
    const uint64_t lo = sl * kMl;
    const uint64_t hi = __umul64hi(sl, kMl) + sl * kMh + sh * kMl;
    const uint64_t nlo = lo + il;
    sh = hi + ih + (nlo < lo ? 1ULL : 0ULL);
    sl = nlo;
    const uint64_t x = sh ^ sl;
    const unsigned rot = (unsigned)(sh >> 58);
    return (x >> rot) | (x << ((64u - rot) & 63u));
  }
  __device__ uint32_t next32() {
    if (has32) { has32 = 0; return u32; }
    const uint64_t v = next64();
    has32 = 1;
    u32 = (uint32_t)(v >> 32);
    return (uint32_t)v;
  }
  __device__ double next_double() { return (double)(next64() >> 11) * (1.0 / 9007199254740992.0); }
  __device__ double standard_normal() {
    constexpr double kR = 3.6541528853610088, kInvR = 0.27366123732975828;
    for (;;) {
      uint64_t r = next64();
      const int idx = (int)(r & 0xff);
      r >>= 8;
      const bool neg = r & 1;
      const uint64_t rabs = (r >> 1) & 0x000fffffffffffffULL;
      double x = (double)rabs * kNpZigWi[idx];
      if (neg) x = -x;
      if (rabs < kNpZigKi[idx]) return x;
      if (idx == 0) {
        for (;;) {
          const double xx = -kInvR * log1p(-next_double());
          const double yy = -log1p(-next_double());
          if (yy + yy > xx * xx) return ((rabs >> 8) & 1) ? -(kR + xx) : kR + xx;
        }
      }
      if ((kNpZigFi[idx - 1] - kNpZigFi[idx]) * next_double() + kNpZigFi[idx] < exp(-0.5 * x * x)) return x;
    }
  }
  __device__ double uniform(double lo, double hi) { return lo + (hi - lo) * next_double(); }
  __device__ int integers(int lo, int hi) {                  // [lo, hi), hi - lo <= 2^32
    const uint32_t rng = (uint32_t)(hi - 1 - lo), excl = rng + 1;
    uint64_t m = (uint64_t)next32() * excl;
    uint32_t left = (uint32_t)m;
    if (left < excl) {
      const uint32_t thr = (0xFFFFFFFFu - rng) % excl;
      while (left < thr) { m = (uint64_t)next32() * excl; left = (uint32_t)m; }
    }
    return lo + (int)(m >> 32);
  }
};

template <typename R>
__device__ __forceinline__ NpPcg64 np_load(const State<R>& S, int e) {
  auto w = [&](int i) { return (uint64_t)S.nprng[(size_t)i * S.fstride + e]; };
  return NpPcg64{w(0) | (w(1) << 32), w(2) | (w(3) << 32), w(4) | (w(5) << 32), w(6) | (w(7) << 32),
                 (uint32_t)w(8), (uint32_t)w(9)};
}
template <typename R>
__device__ __forceinline__ void np_store(const State<R>& S, int e, const NpPcg64& g) {
  const uint32_t v[10] = {(uint32_t)g.sh, (uint32_t)(g.sh >> 32), (uint32_t)g.sl, (uint32_t)(g.sl >> 32),
                          (uint32_t)g.ih, (uint32_t)(g.ih >> 32), (uint32_t)g.il, (uint32_t)(g.il >> 32),
                          g.has32, g.u32};
  for (int i = 0; i < 10; ++i) S.nprng[(size_t)i * S.fstride + e] = v[i];
}

// UsvSimpleEnv.reset (simple_env.py:228-308) with the env's own Generator; usv-asmc-simple also
// zeroes the ASMC state (simple_env_asmc.py:14-16).  Writes the reset obs header into `row`
// (its sensor half, the stale scan, is the caller's).  Draws in double, stored as R.
template <typename R, int MODE>
__device__ void np_reset(const State<R>& S, int e, float* row, R* info = nullptr, int kpath = 0) {
  NpPcg64 g = np_load(S, e);
  const double sx = 0.5 * g.standard_normal() + kBound / 2;                      // :234-235
  const double sy = 0.5 * g.standard_normal() + kBound / 2;
  (void)g.standard_normal(); (void)g.standard_normal(); (void)g.next_double();   // :236-237, discarded
  const double psi = g.uniform(-kPi, kPi);                                       // :238
  const double ang = g.uniform(-kPi, kPi), dist = g.uniform(100, 110);           // :241-242
  const double tx = g.uniform(0, kBound), ty = g.uniform(0, kBound);             // :245
  const double u = g.uniform(0.0, 0.15), v = g.uniform(0.0, 0.15), r = g.uniform(0.0, 0.15);  // :246
  const double mu = g.uniform(1.50, 3);                                          // :249
  (void)g.next_double(); (void)g.next_double();                                  // max_action[1], [2]
  const double mr = g.uniform(3, 6);                                             // :250
  const double refv = g.uniform(0.75, mu);                                       // :251
  const int n = g.integers(15, 30);                                              // :257
  R* ob = S.orow(e);
  const int os = S.ostride;
  int cnt = 0;
  for (int j = 0; j < n; ++j) {                                                  // :258-268
    const double ox = g.uniform(0, kBound), oy = g.uniform(0, kBound);
    if (!(hypot(sx - ox, sy - oy) < 0.5 || hypot(tx - ox, ty - oy) < 0.5)) {
      ob[cnt] = R(ox); ob[os + cnt] = R(oy); ++cnt;
    }
  }
  if (cnt == 0) {                                                                // :270-274
    const double ox = g.uniform(0, kBound), oy = g.uniform(0, kBound);
    ob[0] = R(ox); ob[os] = R(oy); cnt = 1;
  }
  if (kpath > 0) {                                                               // :276-288
    // mag = uniform(0, hypot(*env_bounds) = hypot(0, 20), k); line_x = normal(cos(angle) * mag +
    // path_start[0], 1); line_y likewise: k uniforms, then k normals per axis
    // (the k magnitudes are re-drawn from copies of the generator instead of being buffered)
    const double ca = cos(ang), sa = sin(ang);
    NpPcg64 gx = g, gy = g;
    for (int j = 0; j < kpath; ++j) (void)g.next_double();
    for (int j = 0; j < kpath; ++j) ob[cnt + j] = R((ca * gx.uniform(0, kBound) + sx) + g.standard_normal());
    for (int j = 0; j < kpath; ++j) ob[os + cnt + j] = R((sa * gy.uniform(0, kBound) + sy) + g.standard_normal());
    cnt += kpath;
  }
  for (int j = 0; j < cnt; ++j) ob[2 * os + j] = R(g.uniform(0.15, 0.5));      // :290
  np_store(S, e, g);
  double ps0 = sx, ps1 = sy, pe0 = sx + cos(ang) * dist, pe1 = sy + sin(ang) * dist;   // :243
  double px = sx, py = sy, pp = psi;
  if (const R* X = S.exp) {                                                      // :292-300
    cnt = (int)X[kExpN];
    for (int j = 0; j < cnt; ++j) {
      ob[j] = X[kExpObs + j]; ob[os + j] = X[kExpObs + S.cap + j]; ob[2 * os + j] = X[kExpObs + 2 * S.cap + j];
    }
    ps0 = (double)X[kExpPS]; ps1 = (double)X[kExpPS + 1];
    pe0 = ps0 + cos((double)X[kExpAngle]) * 100; pe1 = ps1 + sin((double)X[kExpAngle]) * 100;
    px = (double)X[kExpPose]; py = (double)X[kExpPose + 1]; pp = (double)X[kExpPose + 2];
  }
  for (int j = cnt; j < S.cap; ++j) { ob[j] = R(0); ob[os + j] = R(0); ob[2 * os + j] = R(0); }
  if (MODE == USV_MODE_ASMC_SIMPLE)
    for (int i = 0; i < kAsmcN; ++i) S.asmc[(size_t)i * S.N + e] = R(0);
  const R x0 = R(px), y0 = R(py), ps = R(pp);
  S.F(F_X)[e] = x0; S.F(F_Y)[e] = y0;
  store_heading<R>(S, e, ps);
  S.F(F_U)[e] = R(u); S.F(F_V)[e] = R(v); S.F(F_R)[e] = R(r);
  S.F(F_PROGRESS)[e] = R(0);
  S.F(F_PX0)[e] = R(ps0); S.F(F_PY0)[e] = R(ps1);
  S.F(F_PX1)[e] = R(pe0); S.F(F_PY1)[e] = R(pe1);
  S.F(F_MAX_U)[e] = R(mu); S.F(F_MAX_R)[e] = R(mr); S.F(F_REF_V)[e] = R(refv);
  S.I(I_NOBS)[e] = cnt;
  S.I(I_ELAPSED)[e] = 0;
  S.I(I_EPISODE)[e] = S.I(I_EPISODE)[e] + 1;
  S.I(I_SCAN)[e] = 0;
  const R angle = wrap_angle(m_atan2(R(ty) - y0, R(tx) - x0) - ps);             // :302, :63-80
  const R dst = m_hypot(x0 - R(tx), y0 - R(ty));
  const R ye = S.exp ? path_ye(x0, y0, R(ps0), R(ps1), R(pe0), R(pe1)) : R(0);
  float h[kHdr];
  make_header<R>(h, R(u), R(v), R(r), angle, dst, ye, R(refv), R(0), R(0), R(mu), R(mr));
  for (int i = 0; i < kHdr; ++i) row[i] = h[i];
  if (info) reset_info<R>(info, x0, y0, ps, R(u), R(v), R(r), R(ps0), R(ps1), R(pe0), R(pe1), ye, cdiv(angle, kPi));
}

// Same-step autoreset in NumPy-exact mode, after the step kernel: envs that ended this step get
// a reset header; their obs row keeps the step's scan as the stale sensors (simple_env.py:302).
template <typename R, int MODE>
__global__ __launch_bounds__(kBlock) void np_autoreset_kernel(State<R> S, IO<R> io) {
  const int e = blockIdx.x * kBlock + threadIdx.x;
  if (e >= S.N || !(io.term[e] | io.trunc[e])) return;
  np_reset<R, MODE>(S, e, io.obs + (size_t)e * kObsDim);
}

// Same-step autoreset with a custom experiment installed (Philox resets): after the step kernel,
// envs that ended this step get the experiment's obstacles, path and pose (simple_env.py:292-300).
template <typename R>
__global__ __launch_bounds__(kBlock) void exp_autoreset_kernel(State<R> S, IO<R> io) {
  const int e = blockIdx.x * kBlock + threadIdx.x;
  if (e >= S.N || !(io.term[e] | io.trunc[e])) return;
  reset_experiment<R>(S, e, S.I(I_EPISODE)[e] - 1, io.obs + (size_t)e * kObsDim, nullptr);
}

// --------------------------------------------------------------------------- UsvAsmc.compute
// The controller on its own (gym_usv/control/usv_asmc.py:53-244), lane per controller: `calls`
// back-to-back compute() calls of 10 substeps each on [n][3] poses / velocities and the [16][n]
// state (asmc_substep's layout).  Same substep functions as the env step; the f32 build applies
// asmc_substep_f32's per-call pose accumulation (10 substeps here, 20 in an env step).
template <typename R>
__global__ __launch_bounds__(kBlock) void asmc_compute_kernel(int n, const R* __restrict__ act, R* pos, R* vel,
                                                              R* st, int* pstep, int perturb, int calls) {
  const int e = blockIdx.x * kBlock + threadIdx.x;
  if (e >= n) return;
  R s[kAsmcN];
#pragma unroll
  for (int i = 0; i < kAsmcN; ++i) s[i] = st[(size_t)i * n + e];
  R x = pos[3 * (size_t)e], y = pos[3 * (size_t)e + 1], psi = pos[3 * (size_t)e + 2];
  R u = vel[3 * (size_t)e], v = vel[3 * (size_t)e + 1], r = vel[3 * (size_t)e + 2];
  const R a0 = act[2 * (size_t)e], a1 = act[2 * (size_t)e + 1];
  int ps = pstep ? pstep[e] : 0;
  const bool pert = perturb != 0;
  for (int c = 0; c < calls; ++c) {
    if constexpr (std::is_same<R, float>::value) {
      float xl = 0.0f, yl = 0.0f, pl = 0.0f;
      const float kt = rintf(psi * 0.159154943f);
      const AsmcRun e0 = asmc_run_begin(s, psi);
      for (int k = 0; k < 10; ++k) asmc_substep_f32(s, a0, a1, x, y, psi, u, v, r, xl, yl, pl, kt, ps + k, pert);
      asmc_run_end(x, y, psi, xl, yl, pl, e0, s);
    } else {
      for (int k = 0; k < 10; ++k) asmc_substep<R>(s, a0, a1, x, y, psi, u, v, r, ps + k, pert);
    }
    ps += 10;                                                   // perturb_step (:199)
  }
#pragma unroll
  for (int i = 0; i < kAsmcN; ++i) st[(size_t)i * n + e] = s[i];
  pos[3 * (size_t)e] = x; pos[3 * (size_t)e + 1] = y; pos[3 * (size_t)e + 2] = psi;
  vel[3 * (size_t)e] = u; vel[3 * (size_t)e + 1] = v; vel[3 * (size_t)e + 2] = r;
  if (pstep) pstep[e] = ps;
}

// --------------------------------------------------------------------------- phase 1
// usv-asmc-simple's two UsvAsmc.compute calls (simple_env_asmc.py:19-25, usv_asmc.py:53-244) on env
// e's pose and velocity, in registers; the ASMC state is loaded and stored here.
template <typename R>
__device__ __forceinline__ void asmc_env_chain(const State<R>& S, int e, int el0, float a_u, float a_r, R& x,
                                               R& y, R& psi, R& u, R& v, R& r, R* psi_d_last = nullptr) {
  // psi_d_last given: row 0 (psi_d_last) is returned there and not stored (the caller rebases it)
  {
    R s[kAsmcN];
#pragma unroll
    for (int i = 0; i < kAsmcN; ++i) s[i] = S.asmc[(size_t)i * S.N + e];
    const R c0 = R(a_u), c1 = R(a_r);
    // perturb_step of the episode's UsvAsmc: 2 compute() x 10 substeps per env step (usv_asmc.py:199)
    const bool pert = S.perturb != 0;
    if constexpr (std::is_same<R, float>::value) {
      float xl = 0.0f, yl = 0.0f, pl = 0.0f;        // position sums, heading compensation (asmc_substep_f32)
      const float kt = rintf(psi * 0.159154943f);    // whole turns of the heading (asmc_substep_f32's J)
      const AsmcRun e0 = asmc_run_begin(s, psi);    // eta_dot_last and psi before the run (asmc_run_end)
      // perturbation hoisted out of the substep loop, so the common loop unrolls (by 4): no
      // loop-carried register rotation (the s[1..3], s[4..9] moves) and the scheduler fills one
      // substep's hazard nops with the next one's independent work (dyn_rec_kernel 13.6 -> 11.4 us
      // at 65 536 envs)
      if (pert) {
        for (int k = 0; k < 20; ++k) asmc_substep_f32(s, c0, c1, x, y, psi, u, v, r, xl, yl, pl, kt, 20 * el0 + k, true);
      } else {
#pragma unroll 4
        for (int k = 0; k < 20; ++k) asmc_substep_f32(s, c0, c1, x, y, psi, u, v, r, xl, yl, pl, kt, 0, false);
      }
      asmc_run_end(x, y, psi, xl, yl, pl, e0, s);
    } else {
      if (pert) {
        for (int k = 0; k < 20; ++k) asmc_substep<R>(s, c0, c1, x, y, psi, u, v, r, 20 * el0 + k, true);
      } else {
#pragma unroll 4
        for (int k = 0; k < 20; ++k) asmc_substep<R>(s, c0, c1, x, y, psi, u, v, r, 0, false);
      }
    }
#pragma unroll
    for (int i = psi_d_last ? 1 : 0; i < kAsmcN; ++i) S.asmc[(size_t)i * S.N + e] = s[i];
    if (psi_d_last) *psi_d_last = s[0];
  }
}

// UsvSimpleEnv.step kinematics..reward terms (simple_env.py:310-346); for usv-asmc-simple
// first 2x UsvAsmc.compute (simple_env_asmc.py:18-27) and then step(zeros(2)).
// Also returns sin/cos of the new heading so the wave-per-env lidar does not recompute them.
// CHAIN = false (usv-asmc-simple only): asmc_chain_kernel already ran the two compute() calls and
// stored the pose and velocity they left; this is then UsvSimpleEnv.step(zeros(2)) on them.
template <typename R, int MODE, bool CHAIN = true>
__device__ void env_dynamics(const State<R>& S, int e, float a_u, float a_r, float (&hdr)[kHdr],
                             R& px, R& py, R& psp, R& pcp, R& partial, bool& trunc, R* info = nullptr) {
  R x = S.F(F_X)[e], y = S.F(F_Y)[e], psi = S.F(F_PSI)[e];
  R u = S.F(F_U)[e], v = S.F(F_V)[e], r = S.F(F_R)[e];
  const int el0 = S.I(I_ELAPSED)[e];
  constexpr bool kF32 = std::is_same<R, float>::value;
  constexpr bool kAsmc = MODE == USV_MODE_ASMC_SIMPLE;
  int k0 = 0;                                        // f32: the heading's whole turns (store_heading)
  R pdl = R(0);                                      // f32 usv-asmc-simple: psi_d_last, phi's frame
  if constexpr (kF32) {
    k0 = S.I(I_TURNS)[e];
    if constexpr (kAsmc && !CHAIN) pdl = S.asmc[e];
  }
  // every load of the step before its first store (the state stores go out early, below): with one
  // in-order vmcnt counter a load issued after a store returns only once that store is acknowledged
  const R lu = S.F(F_LAST_U)[e], lr = S.F(F_LAST_R)[e];
  const R mu = S.F(F_MAX_U)[e], mr = S.F(F_MAX_R)[e], refv = S.F(F_REF_V)[e];
  const R x0 = S.F(F_PX0)[e], y0 = S.F(F_PY0)[e];
  const R x1 = S.F(F_PX1)[e], y1 = S.F(F_PY1)[e];
  const R prog0 = S.F(F_PROGRESS)[e];
  if (kAsmc) {
    if constexpr (CHAIN) asmc_env_chain<R>(S, e, el0, a_u, a_r, x, y, psi, u, v, r, kF32 ? &pdl : nullptr);
    a_u = 0.0f;                                                                   // step(zeros(2))
    a_r = 0.0f;
  }
  // action = max_action * insert(action, 1, 0); filtered 0.8/0.2 (:311-317)
  const R a3u = R(0.8) * lu + R(0.2) * (mu * R(a_u));
  const R a3r = R(0.8) * lr + R(0.2) * (mr * R(a_r));
  // per-step acceleration clip, then speed clip; max_action[1] = 0 pins v to 0 (:320-321)
  const R dvu = m_clip(a3u - u, R(-kMaxAccU), R(kMaxAccU));
  const R dvr = m_clip(a3r - r, R(-kMaxAccR), R(kMaxAccR));
  u = m_clip(u + dvu, -mu, mu);
  v = R(0);
  r = m_clip(r + dvr, -mr, mr);
  R sp, cp;
  fx_sincos(psi, &sp, &cp);
  x = x + (u * cp) * R(kDt);                                                      // :322-324
  y = y + (u * sp) * R(kDt);
  psi = psi + r * R(kDt);
  // _get_closest_point (:139-148)
  const R dx = x1 - x0, dy = y1 - y0;
  const R det = dx * dx + dy * dy;
  R a = dyn_div(dy * (y - y0) + dx * (x - x0), det);
  a = a + R(kLookahead);
  a = m_clip(a, prog0, R(1));
  const int el = el0 + 1;
  // the state stores, as soon as the new state exists (their acknowledgements then overlap the rest
  // of phase 1; a same-step reset by another wave orders itself after them: step_q_body)
  {
    R ps = psi;
    if constexpr (kF32) {                            // the rebase (see the heading representation)
      // branch-free and stored unconditionally (n = 0 leaves both values unchanged, bit for bit): a
      // conditional store made the compiler sink the k0 load into its branch, and a wave with one
      // rebasing lane then waited a memory round trip in the middle of phase 1
      const float n = turns_of(psi);
      ps = sub_turns(psi, n);
      S.I(I_TURNS)[e] = k0 + (int)n;
      if constexpr (kAsmc) S.asmc[e] = sub_turns(pdl, n);   // (the chain left row 0 to this store)
    }
    S.F(F_X)[e] = x; S.F(F_Y)[e] = y; S.F(F_PSI)[e] = ps;
    S.F(F_U)[e] = u; S.F(F_V)[e] = v; S.F(F_R)[e] = r;
    S.F(F_LAST_U)[e] = a3u; S.F(F_LAST_R)[e] = a3r;
    S.F(F_PROGRESS)[e] = a;
    S.I(I_ELAPSED)[e] = el;
    S.I(I_SCAN)[e] = 1;
  }
  const R tx = x0 + a * dx, ty = y0 + a * dy;
  // _get_ye (:133-137): sin/cos of the path angle a_k = atan2(dy, dx) are dy/|d|, dx/|d|
  const R inv_len = dyn_div(R(1), dyn_sqrt(det));
  const R sak = dy * inv_len, cak = dx * inv_len;
  const R ye = -(x - x0) * sak + (y - y0) * cak;
  // _get_angle_to_target (:67-69), distance (:74)
  const R angle = wrap_angle(fx_atan2(ty - y, tx - x) - psi);
  const R ddx = x - tx, ddy = y - ty;
  const R dist = dyn_sqrt(ddx * ddx + ddy * ddy);
  trunc = (x > R(kBound)) | (x < R(0)) | (y > R(kBound)) | (y < R(0)) |   // :336
          (S.limit > 0 && el >= S.limit);                                 // TimeLimit
  make_header<R>(hdr, u, v, r, angle, dist, ye, refv, lu, lr, mu, mr);   // obs uses PREVIOUS action
  // _get_reward without the collision term (:150-186)
  const R dact = m_abs(lu - a3u) + m_abs(lr - a3r);
  const R yk = cdiv(ye, kYeK);
  const R e1 = fx_exp(-m_abs(yk)), e2 = fx_exp(-(yk * yk));
  const R ye_r = e1 > e2 ? e1 : e2;
  const R ang_r = fx_exp(-m_abs(angle));
  const R vel_r = fx_exp(-m_abs(dyn_sqrt(u * u + v * v) - refv)) * R(0.05);
  const R dact_r = -(dact / R(2)) * R(0.15);
  partial = ye_r + ang_r + vel_r + dact_r;
  if (info) {                                        // _get_info + reward_info (:102-115, :189-199)
    const R vals[USV_INFO_DIM] = {x, y, heading_abs(psi, k0), u, v, r,
                                  x0, y0, x1, y1, a3u, a3r, ye,
                                  cdiv(angle, kPi), ye_r, ang_r, dact_r, dact, vel_r, refv, lu, lu - refv};
#pragma unroll
    for (int i = 0; i < USV_INFO_DIM; ++i) info[i] = vals[i];
  }
  px = x; py = y;
  heading_sincos(psi, &psp, &pcp);
}

// --------------------------------------------------------------------------- lidar
// 128-ray lidar of one env at pose (px, py, heading sin/cos), wave-per-env.  Lane l owns rays
// l and l+64; lane j holds obstacle j (`o`).  Restates compute_sensor_measurments /
// compute_obstacle_positions / _compute_sensor_distances (usv_asmc_ca_env.py:411-461,
// 500-519): per ray, the hit obstacle with the smallest key d_j = |c_j - p| - r_j, which is
// the reference's first hit in argsort(d) order.  Every product is an explicit fma or a
// rounded multiply and every variant evaluates the identical per-(ray, obstacle) arithmetic,
// so all variants -- and the step and reset kernels -- produce bit-identical scans.
template <typename R> struct Ray { R c, s, bk; int bj; };

template <typename R> __device__ __forceinline__ R l_sqrt(R x) { return m_sqrt(x); }
template <> __device__ __forceinline__ float l_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
template <typename R> __device__ __forceinline__ R l_norm(R x) { return x / R(kSensorMax); }
template <> __device__ __forceinline__ float l_norm(float x) { return x * 0.01f; }

// Ray frame.  Obstacles are rotated once into the frame of ray 0 (heading - 120 deg): a along
// ray 0, b to its left; ray i is then (cos i*res, sin i*res) from the table, and for every
// (ray, obstacle) pair proj = a cos + b sin, perp = a sin - b cos -- the reference's projection
// (usv_asmc_ca_env.py:506-518) with both vectors in that frame, so no per-pair rotation.
template <typename R> __device__ __forceinline__ R ray_c(R cp, R sp, R co, R so) { return m_fma(cp, co, -(sp * so)); }
template <typename R> __device__ __forceinline__ R ray_s(R cp, R sp, R co, R so) { return m_fma(sp, co, cp * so); }
template <typename R> __device__ __forceinline__ void to_ray0(R dx, R dy, R c0, R s0, R& a, R& b) {
  a = m_fma(dx, c0, dy * s0);
  b = m_fma(dy, c0, -(dx * s0));
}

template <typename R, bool RANGE_CHECK>
__device__ __forceinline__ void ray_pair(Ray<R>& ra, R jdx, R jdy, R jr2, R jk, int j) {
  const R proj = m_fma(jdx, ra.c, jdy * ra.s);    // obstacle x in the ray frame (:506-517)
  const R perp = m_fma(jdx, ra.s, -(jdy * ra.c)); // obstacle y, mirrored (:518)
  const R delta = m_fma(-perp, perp, jr2);        // r^2 - y^2 (:453)
  bool hit = (proj >= R(0)) & (delta >= R(0)) & (jk < ra.bk);
  if (RANGE_CHECK) hit = hit && (proj - l_sqrt(delta)) < R(kSensorMax);   // :458
  ra.bk = hit ? jk : ra.bk;
  ra.bj = hit ? j : ra.bj;
}

// Lidar variants (compile-time): bit 0 = drop obstacles wholly inside the rear blind sector
// before the ray loop, bit 1 = obstacle loop unrolled by two, bit 2 = angular-window pair
// expansion (f32: lidar_window / lidar_window2; f64: lidar_window_d).  The max-range test of :458 runs only in waves with an
// obstacle >= 99 m away (wave-uniform template switch).
constexpr int kLidSkip = 1, kLidUnroll2 = 2, kLidWindow = 4;

template <typename R, bool RANGE_CHECK, bool UNROLL2>
__device__ __forceinline__ void ray_loop(Ray<R>& r0, Ray<R>& r1, R dx, R dy, R r2, R key, int n) {
  if (UNROLL2) {
    for (int j = 0; j < n; j += 2) {             // n even (padded with a never-hit obstacle)
      const R adx = bcast(dx, j), ady = bcast(dy, j), ar2 = bcast(r2, j), ak = bcast(key, j);
      const R bdx = bcast(dx, j + 1), bdy = bcast(dy, j + 1), br2 = bcast(r2, j + 1), bk = bcast(key, j + 1);
      ray_pair<R, RANGE_CHECK>(r0, adx, ady, ar2, ak, j);
      ray_pair<R, RANGE_CHECK>(r1, adx, ady, ar2, ak, j);
      ray_pair<R, RANGE_CHECK>(r0, bdx, bdy, br2, bk, j + 1);
      ray_pair<R, RANGE_CHECK>(r1, bdx, bdy, br2, bk, j + 1);
    }
  } else {
    for (int j = 0; j < n; ++j) {                // n wave-uniform: scalar loop, v_readlane bcast
      const R jdx = bcast(dx, j), jdy = bcast(dy, j), jr2 = bcast(r2, j), jk = bcast(key, j);
      ray_pair<R, RANGE_CHECK>(r0, jdx, jdy, jr2, jk, j);
      ray_pair<R, RANGE_CHECK>(r1, jdx, jdy, jr2, jk, j);
    }
  }
}

template <typename R>
__device__ __forceinline__ R reading_of(R c, R s, int bj, R dx, R dy, R r2) {
  const int src = bj < 0 ? 0 : bj;
  const R gdx = __shfl(dx, src, kWave), gdy = __shfl(dy, src, kWave), gr2 = __shfl(r2, src, kWave);
  const R proj = m_fma(gdx, c, gdy * s);
  const R perp = m_fma(gdx, s, -(gdy * c));
  const R delta = m_fma(-perp, perp, gr2);
  return bj >= 0 ? proj - l_sqrt(delta) : R(kSensorMax);                        // :457-459
}

// Rays span [psi - 120deg, psi + 118.125deg]; the blind sector between them has half-width
// 60.9375deg around psi + 179.0625deg.  An obstacle (distance d > r) can be hit by no ray if
// its angular extent [phi - a, phi + a], a = asin(r/d), lies inside that sector with a
// 2-ray (3.75deg) margin:  dot(c - p, w) > cos(h)*sqrt(d^2 - r^2) + sin(h)*r  and r < d*sin(h)
// with h = 57.1875deg.  Skipping such obstacles never changes a reading.
constexpr double kBlindC = -0.99985057700379, kBlindS = 0.01636173162648;  // cos/sin(179.0625deg)
constexpr double kBlindCosH = 0.54212310917132, kBlindSinH = 0.84029769328406;  // h = 57.1875deg
constexpr double kRes = (4.0 * kPi / 3.0) / kSensors;
constexpr double kStartC = -0.5, kStartS = -0.86602540378443865;                 // cos/sin(-120deg)

// Per-env lidar outputs: readings of this lane's two rays and the three wave-uniform flags the
// step needs (simple_env.py:153-155, :334; the "< max range" test of :458 only matters if an
// obstacle is ~100 m away).
template <typename R> struct Scan { R rd0, rd1; bool term, far; };

// |atan2(y, x)| error < 7e-4 rad = 0.02 ray (degree-5 minimax on [0,1] + octant folding), well inside
// the quarter-ray window margin; only used to size the conservative ray windows, never for a reading.
// atan2 to |err| <= 6.1e-4 rad (degree-5 odd minimax on [0, 1] plus octant folding)
__device__ __forceinline__ float fast_atan2(float y, float x) {
  const float ax = fabsf(x), ay = fabsf(y);
  const float mx = fmaxf(fmaxf(ax, ay), 1e-30f), mn = fminf(ax, ay);
  const float t = mn * __builtin_amdgcn_rcpf(mx);
  const float s = t * t;
  float p = fmaf(fmaf(0.0793406442f, s, -0.288691819f), s, 0.995358229f) * t;
  p = ay > ax ? 1.57079633f - p : p;
  p = x < 0.0f ? 3.14159265f - p : p;
  return y < 0.0f ? -p : p;
}

constexpr double kWinMargin = 0.05;   // ray-window margin of the window lidar, in rays (lidar_window)
// armed (no-hit) slot of lidar_window2: key bits all ones (above every ord_key of a finite or
// infinite key, so any hit wins the ds_min_u64) and reading bits of the max range 100.0f
constexpr unsigned long long kSlotArm = 0xFFFFFFFF42C80000ull;
static_assert(kSensorMax == 100.0, "kSlotArm's reading half is 100.0f");

__device__ __forceinline__ unsigned ord_key(float k) {   // float -> order-preserving uint
  const unsigned u = __float_as_uint(k);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Exclusive prefix from an inclusive one: the value of lane l - 1 (DPP wave_shr:1; lane 0 gets 0).
__device__ __forceinline__ int wave_excl_of(int incl) {
  return __builtin_amdgcn_update_dpp(0, incl, 0x138, 0xF, 0xF, true);
}
// Inclusive prefix sum over the 64 lanes (DPP row scans + row carries).
__device__ __forceinline__ int wave_incl_scan(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true);   // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true);   // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true);   // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true);   // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
  return v;
}

template <typename R, int LID>
__device__ __forceinline__ void lidar_brute(R dx, R dy, R r2, R key, R d, R rr, bool valid, int n,
                                            bool far, R sp, R cp, R co0, R so0, R co1, R so1,
                                            Scan<R>& out) {
  const int l = lane_id();
  int m = n;
  R a, b;
  to_ray0(dx, dy, ray_c(cp, sp, R(kStartC), R(kStartS)), ray_s(cp, sp, R(kStartC), R(kStartS)), a, b);
  if (LID & kLidSkip) {
    const R wx = cp * R(kBlindC) - sp * R(kBlindS), wy = sp * R(kBlindC) + cp * R(kBlindS);
    const R dot = dx * wx + dy * wy;
    const R lim = R(kBlindCosH) * l_sqrt(m_abs(d * d - rr * rr)) + R(kBlindSinH) * rr;
    const bool blind = (d > rr) & (rr < d * R(kBlindSinH)) & (dot > lim);
    const bool keep = valid & !blind;
    // stream-compact the kept obstacles (order preserved, so min-key ties still resolve to
    // the lowest original index)
    const unsigned long long ball = ballot(keep);
    m = __popcll(ball);
    const int pos = __builtin_amdgcn_mbcnt_hi((unsigned)(ball >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)ball, 0));
    const int dst = keep ? pos : 63;               // dropped lanes all land in lane 63 (unused)
    a = __builtin_bit_cast(R, permute(dst, __builtin_bit_cast(typename Bits<R>::T, a)));
    b = __builtin_bit_cast(R, permute(dst, __builtin_bit_cast(typename Bits<R>::T, b)));
    r2 = __builtin_bit_cast(R, permute(dst, __builtin_bit_cast(typename Bits<R>::T, r2)));
    key = __builtin_bit_cast(R, permute(dst, __builtin_bit_cast(typename Bits<R>::T, key)));
  }
  if (LID & kLidUnroll2) {
    if (l >= m) { r2 = R(-1); key = big<R>(); }    // padding obstacle: delta < 0, never hit
    m = (m + 1) & ~1;
  }
  Ray<R> r0{co0, so0, big<R>(), -1};
  Ray<R> r1{co1, so1, big<R>(), -1};
  if (!far) ray_loop<R, false, (LID & kLidUnroll2) != 0>(r0, r1, a, b, r2, key, m);
  else ray_loop<R, true, (LID & kLidUnroll2) != 0>(r0, r1, a, b, r2, key, m);
  out.rd0 = reading_of(r0.c, r0.s, r0.bj, a, b, r2);
  out.rd1 = reading_of(r1.c, r1.s, r1.bj, a, b, r2);
}

// Angular-window lidar (f32).  Lane j computes the ray-index windows its obstacle can touch
// (conservative: a quarter ray of margin around an upper bound of asin(r/d), pi/2 when the boat is
// inside it), the (obstacle, ray) pairs are expanded over the lanes (prefix sum; each pair's
// owner found with LDS start markers and a max-scan), each pair runs the same exact test as
// the brute loop, and the hit with the smallest key per ray wins through an LDS ds_min_u64 on
// (order-preserving key bits << 32 | hit distance bits) -- the min-key rule, and the winner's
// reading rides along as the payload.  Bit-identical to lidar_brute except on an exact key tie
// between two different obstacles (measure zero; brute then takes the lower index, this the
// nearer hit, and the reference's own argsort tie order is unspecified).  ~50 pair tests per
// env instead of 128 x n.
struct WinLds {
  unsigned long long* slot;   // [128] per wave, ~0 between envs
  int* mark;                  // [64]  per wave (cross-lane through LDS: ordered by a wave fence)
  const float2* rayoff;       // [128] block-shared ray offset table
};

// One env's obstacle row in LDS: the x, y, r planes (the global row copied verbatim by LDS-DMA,
// or staged through registers by the reset kernel).
template <typename R> struct RowSoA {
  const R* x; const R* y; const R* r;
  __device__ __forceinline__ void get(int j, R& X, R& Y, R& Rr) const { X = x[j]; Y = y[j]; Rr = r[j]; }
};

// Inclusive max-scan over the 64 lanes of non-negative values (DPP row scans + row_bcast
// carries; identity 0, so bound_ctrl zero-fill folds each step into one v_max_i32_dpp).
__device__ __forceinline__ int wave_incl_max(int v) {
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true));   // row_shr:1
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true));   // row_shr:2
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true));   // row_shr:4
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true));   // row_shr:8
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false));  // row_bcast:15
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false));  // row_bcast:31
  return v;
}

// The same scan as fused DPP maxes in one asm block: a lane whose row is masked off by row_bcast keeps
// its value (vdst = src1), so no zero-filled temporaries are needed.  s_nop 1 before each DPP read
// of the VGPR the previous VALU wrote (gfx9 DPP hazard).
// floor(x) converted to int in one instruction (|x| well inside the int range here)
__device__ __forceinline__ int cvt_flr_i32(float x) {
  int r;
  asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

__device__ __forceinline__ int wave_incl_max_asm(int v) {
  asm volatile("s_nop 1\n\t"
               "v_max_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 1\n\t"
               "v_max_i32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 1\n\t"
               "v_max_i32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 1\n\t"
               "v_max_i32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 1\n\t"
               "v_max_i32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\ts_nop 1\n\t"
               "v_max_i32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf"
               : "+v"(v));
  return v;
}

// Two independent max-scans interleaved in one asm block: each DPP read of a VGPR the previous
// VALU wrote needs two wait states, here the other chain's instruction plus one s_nop 0.
__device__ __forceinline__ void wave_incl_max2_asm(int& a, int& b) {
  asm volatile("s_nop 1\n\t"
               "v_max_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
               "v_max_i32_dpp %1, %1, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 0\n\t"
               "v_max_i32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
               "v_max_i32_dpp %1, %1, %1 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 0\n\t"
               "v_max_i32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
               "v_max_i32_dpp %1, %1, %1 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 0\n\t"
               "v_max_i32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
               "v_max_i32_dpp %1, %1, %1 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\ts_nop 0\n\t"
               "v_max_i32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
               "v_max_i32_dpp %1, %1, %1 row_bcast:15 row_mask:0xa bank_mask:0xf\n\ts_nop 0\n\t"
               "v_max_i32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
               "v_max_i32_dpp %1, %1, %1 row_bcast:31 row_mask:0xc bank_mask:0xf"
               : "+v"(a), "+v"(b));
}

template <bool RANGE_CHECK, typename Row>
__device__ __forceinline__ void lidar_window(float dx, float dy, float key, float d, float rr, bool valid,
                                             float px, float py, float sp, float cp, const WinLds& L,
                                             const Row& row, Scan<float>& out) {
  const int l = lane_id();
  const float c0r = ray_c(cp, sp, (float)kStartC, (float)kStartS);
  const float s0r = ray_s(cp, sp, (float)kStartC, (float)kStartS);
  float a, b;
  to_ray0(dx, dy, c0r, s0r, a, b);
  const float phi = fast_atan2(b, a);                 // CCW angle from ray 0; ray i at i*res
  // |err| of the window edges: fast_atan2 <= 6.1e-4 rad (0.019 ray), float rounding ~1e-6 rad; a
  // ray 1e-5 rad outside the true extent already fails the exact test by ~r*d*1e-5 >> ulp.  The
  // margin (0.05 ray = 1.6e-3 rad) covers both 2.6x over.
  const float margin = (float)(kWinMargin * kRes);
  const bool inside = d <= rr * 1.001f;
  // asin(x) <= x + (pi/2 - 1) x^3 on [0, 1] (Taylor coefficients >= 0 summing to pi/2 at x = 1)
  const float x = fminf(rr * __builtin_amdgcn_rcpf(d), 1.0f);
  const float half = inside ? (float)(kPi / 2) + margin
                            : fmaf((float)(kPi / 2 - 1) * x, x * x, x) + margin;
  // in ray units; the second window is the first shifted by one turn = 2 pi / res = 192 rays
  // exactly (rounding of the shifted float edges would only move an edge that lies within
  // ~1e-5 ray of an integer, i.e. well inside the quarter-ray margin)
  const float inv = (float)(1.0 / kRes);
  const float pr = phi * inv, hr = half * inv;
  const int a1 = (int)ceilf(pr - hr), b1 = (int)floorf(pr + hr);
  static_assert(kSensors * 3 == 2 * 192, "192 rays per turn");
  const int lo1 = max(0, a1), hi1 = min(127, b1);
  const int lo2 = max(0, a1 + 192), hi2 = min(127, b1 + 192);
  const int len1 = valid ? max(0, hi1 - lo1 + 1) : 0, len2 = valid ? max(0, hi2 - lo2 + 1) : 0;
  const int cnt = len1 + len2;
  const int incl = wave_incl_scan(cnt);
  const int off = incl - cnt;
  const int W = __builtin_amdgcn_readlane(incl, 63);
  const int meta = lo1 | (len1 << 8) | (lo2 << 16);
  const unsigned ok = ord_key(key);
  int carry = 0;                                      // owner marks are lane + 1; 0 = none
  for (int base = 0; base < W; base += kWave) {       // wave-uniform pass count
    // owner of pair q = base + l: the obstacle whose run of pairs starts at or before q
    L.mark[l] = 0;
    if (cnt > 0 && off >= base && off < base + kWave) L.mark[off - base] = l + 1;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");   // other lanes' marks must be read
    __builtin_amdgcn_wave_barrier();
    const int j1 = max(wave_incl_max(L.mark[l]), carry);
    carry = __builtin_amdgcn_readlane(j1, 63);
    const int j = j1 - 1;
    const int q = base + l;
    const int jj = j < 0 ? 0 : j;
    const int k = q - __shfl(off, jj, kWave);
    const int mj = __shfl(meta, jj, kWave);
    const unsigned gk = (unsigned)__shfl((int)ok, jj, kWave);
    const int l1 = mj & 255, n1 = (mj >> 8) & 255, l2 = mj >> 16;
    const int i = min(max((k < n1 ? l1 : l2 - n1) + k, 0), 127);
    float gx, gy, gr, ga, gb;
    row.get(jj, gx, gy, gr);
    to_ray0(gx - px, gy - py, c0r, s0r, ga, gb);
    const float2 cs = L.rayoff[i];
    const float proj = fmaf(ga, cs.x, gb * cs.y);
    const float perp = fmaf(ga, cs.y, -(gb * cs.x));
    const float delta = fmaf(-perp, perp, gr * gr);
    const float dist = proj - l_sqrt(delta);                 // reading if this pair wins (:457)
    bool hit = (q < W) & (proj >= 0.0f) & (delta >= 0.0f);
    if (RANGE_CHECK) hit = hit && dist < (float)kSensorMax;   // :458
    if (hit)
      atomicMin(&L.slot[i], ((unsigned long long)gk << 32) | __float_as_uint(dist));
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");     // all lanes' ds_min_u64 landed
  __builtin_amdgcn_wave_barrier();
  const unsigned long long v0 = L.slot[l], v1 = L.slot[l + 64];
  L.slot[l] = kSlotArm;                               // re-arm for this wave's next env
  L.slot[l + 64] = kSlotArm;
  out.rd0 = __uint_as_float((unsigned)v0);           // no hit: the armed payload, max range
  out.rd1 = __uint_as_float((unsigned)v1);
}

// Two envs per wave (f32 window path, <= 32 obstacles each): lanes 0..31 hold env A's
// obstacles, lanes 32..63 env B's, both envs' (obstacle, ray) pairs go into ONE expanded list,
// and each pair takes the pose of its owner's env.  The per-obstacle setup, the scans and the
// pass overhead are shared by the two envs; each pair runs the identical exact test, so the
// readings are bit-identical to one-env-per-wave.  Slots [256]: env A rays, then env B rays.
//
// The obstacle lanes leave (a, b, r^2, key bits) records in the rows buffer (lane j at slot j;
// written after every lane's row reads, which the wave's LDS instructions complete in order),
// and each pair reads its owner's record: no pose select, no rotation and no re-read of the row.
// Each lane brings its own env's ray-0 direction (c0r, s0r) = (cos, sin)(psi - 120 deg).
// One ray window per obstacle: phi is taken in [-32.5, 159.5) rays from ray 0, i.e. with the branch
// cut in the middle of the rear blind sector (rays cover [0, 127], the blind sector (127, 192)), so a
// window of half-width < 32.5 rays never wraps onto the rays; wider ones (an obstacle closer than
// r / sin(61 deg), or the boat inside it) take all 128 rays, the exact test sorting them out.
// `far` (wave-uniform): some obstacle is >= 99 m away, where the reference's `< max range` test
// (usv_asmc_ca_env.py:458) can matter; it is applied to every pair then.
// rotA / rotB (wave-uniform, 0..63): lane l receives env A's readings of rays (l - rotA) & 63 and
// 64 + ((l - rotA) & 63) (env B likewise with rotB), i.e. the scan rotated across lanes for free (the
// slot reads take the rotated addresses); the block-queue step stores an env pair's obs rows as
// 32-B-aligned spans this way.
__device__ __forceinline__ void lidar_window2(float dx, float dy, float key, float d, float rr, bool valid, bool far,
                                              float c0r, float s0r, float4* rec, const WinLds& L, int* mark2,
                                              Scan<float>& A, Scan<float>& B, QProf* qp = nullptr,
                                              int rotA = 0, int rotB = 0, int* wout = nullptr) {
  const int l = lane_id();
  float a, b;
  to_ray0(dx, dy, c0r, s0r, a, b);
  const float inv = (float)(1.0 / kRes);
  float pr = fast_atan2(b, a) * inv;                  // CCW angle from ray 0 in rays, (-96, 96]
  pr = pr < -32.5f ? pr + 192.0f : pr;                // -> [-32.5, 159.5)
  const float margin = (float)(kWinMargin * kRes);    // see lidar_window
  const float x = fminf(rr * __builtin_amdgcn_rcpf(d), 1.0f);
  // asin(x) <= x + (pi/2 - 1) x^3 (see lidar_window); boat inside: all rays
  const float hr = (fmaf((float)(kPi / 2 - 1) * x, x * x, x) + margin) * inv;
  // all rays when the window reaches 32 rays: that includes the boat inside the obstacle (x = 1
  // gives hr = 32.05), and a narrower window never wraps onto the rays.  ceil(v) = -floor(-v)
  // (v_cvt_flr_i32_f32: floor and convert in one instruction)
  const bool wide = hr >= 32.0f;
  // both converts unconditionally (the conversion saturates on a wide window's large operands): with a
  // convert inside each select arm the compiler branches on exec around it, twice per env pair
  const int flo = cvt_flr_i32(hr - pr), fhi = cvt_flr_i32(pr + hr);
  const int lo = wide ? 0 : max(0, -flo);
  const int hi = wide ? 127 : min(127, fhi);
  const int cnt = valid ? max(0, hi - lo + 1) : 0;
  const int incl = wave_incl_scan(cnt);
  const int off = wave_excl_of(incl);
  const int W = __builtin_amdgcn_readlane(incl, 63);
  if (wout) *wout = W;                                 // (diagnostic builds: the pair's window size)
  // Segment marks: obstacle lane l's run of pairs starts at off and maps pair q to slot
  // q + (lo - off) + 128 [env B], i.e. ray (slot & 127).  Its mark, written at off, is
  // l << 16 | (lo - off + 128 [env B] + 32768): the owner in the high bits keeps the max-scan in
  // run order and the slot offset rides in the low bits (in [24704, 33023]), so a pair finds its
  // owner, its ray and its slot from one max-scan, with no per-pair gather of the owner's window.
  // A cleared mark is 0, below every mark (the low bits are > 0), and pair 0 always has one (the
  // first obstacle with pairs starts at 0), so every pair's scan result names an owner.
  const int mk0 = (l << 16) | (lo - off + (l >= 32 ? 128 : 0) + 32768);
  rec[l] = make_float4(a, b, rr * rr, __uint_as_float(ord_key(key)));
  // The marks are cleared once per call (below), not per pass: a mark left by an earlier pass of
  // this call is <= that pass's carry, which the max-scan folds in anyway.
  // the pass that holds this obstacle's mark (-1: no pairs) and the mark's index in it
  const int mpass = cnt > 0 ? off >> 6 : -1;
  int* const mslot = L.mark + (off & (kWave - 1));
  int carry = 0;
  QMARK(2);
  // pair q = base + l of a pass whose max-scanned mark is mk: owner, ray, exact test, ds_min.
  // pair_ld reads the owner's record and the ray, pair_do tests and takes the ds_min; the two-pass
  // case issues both passes' reads before either test (one LDS round trip for both).
  struct PairIn { float4 o; float2 cs; int si; };
  auto pair_ld = [&](int base, int mk) {
    const int jj = mk >> 16;                          // owner obstacle lane
    // slot of (owner env, ray) of pair q = base + l: q + (mk & 0xffff) - 32768, of which only the
    // low 8 bits are used (= those of q + mk); exact for q < W, other lanes (no hit) read some
    // ray's offsets
    const int si = base + l + mk;
    return PairIn{rec[jj], L.rayoff[si & 127], si};   // owner's (a, b, r^2, key bits), ray (cos, sin)
  };
  auto pair_do = [&](int base, const PairIn& p) {
    const float4 o = p.o;
    const float2 cs = p.cs;
    // the key half of the payload before the hit branch (the whole record is read by one
    // ds_read_b128: the key is not re-read inside the branch)
    unsigned long long* const sl = &L.slot[p.si & 255];
    const unsigned kb = __float_as_uint(o.w);
    asm volatile("" :: "v"(kb));
    const float proj = fmaf(o.x, cs.x, o.y * cs.y);
    const float perp = fmaf(o.x, cs.y, -(o.y * cs.x));
    const float delta = fmaf(-perp, perp, o.z);
    const float dist = proj - l_sqrt(delta);
    const bool hit = (l < W - base) & (proj >= 0.0f) & (delta >= 0.0f) & (!far | (dist < (float)kSensorMax));  // :458
    if (hit)                                          // slots: env A's rays, then env B's
      atomicMin(sl, ((unsigned long long)kb << 32) | __float_as_uint(dist));
  };
  auto pair = [&](int base, int mk) { pair_do(base, pair_ld(base, mk)); };
  int base = 0, pass = 0;
  if (W > kWave) {
    // passes 0 and 1 at once (1.65 passes per env pair on average at C3): pass 1's marks go to mark2, 64 ints
    // that no DMA touches (the tail of the row buffer the next pair's 768 B of rows land in; it
    // held records last time, so it is cleared first -- LDS ops of a wave complete in order),
    // and the two max-scans run interleaved; pass 1's carry is pass 0's last mark (18.88 -> 18.70 us
    // per step at 65 536 envs, tools/exp_step_ab.sh)
    QCOUNT(9, 2);
    mark2[l] = 0;
    if (mpass == 0) *mslot = mk0;
    if (mpass == 1) mark2[off & (kWave - 1)] = mk0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");   // marks and records visible
    __builtin_amdgcn_wave_barrier();
    int m0 = L.mark[l], m1 = mark2[l];
    wave_incl_max2_asm(m0, m1);
    m1 = max(m1, __builtin_amdgcn_readlane(m0, 63));
    carry = __builtin_amdgcn_readlane(m1, 63);
    const PairIn p0 = pair_ld(0, m0), p1 = pair_ld(kWave, m1);
    pair_do(0, p0);
    pair_do(kWave, p1);
    base = 2 * kWave;
    pass = 2;
  }
  for (; base < W; base += kWave, ++pass) {           // wave-uniform pass count
    QCOUNT(9, 1);
    if (mpass == pass) *mslot = mk0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");   // marks and records visible
    __builtin_amdgcn_wave_barrier();
    const int mk = max(wave_incl_max_asm(L.mark[l]), carry);
    carry = __builtin_amdgcn_readlane(mk, 63);
    pair(base, mk);
  }
  QMARK(3);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");     // all lanes' ds_min_u64 landed
  __builtin_amdgcn_wave_barrier();
  const int la = (l - rotA) & (kWave - 1), lb = (l - rotB) & (kWave - 1);
  const unsigned long long a0 = L.slot[la], a1s = L.slot[la + 64];
  const unsigned long long b0 = L.slot[128 + lb], b1s = L.slot[192 + lb];
  // re-arm for this wave's next pair (after every lane's reads: a wave's LDS ops complete in order)
  L.slot[l] = kSlotArm; L.slot[l + 64] = kSlotArm;
  L.slot[128 + l] = kSlotArm; L.slot[192 + l] = kSlotArm;
  L.mark[l] = 0;
  A.rd0 = __uint_as_float((unsigned)a0);              // no hit: the armed payload, max range
  A.rd1 = __uint_as_float((unsigned)a1s);
  B.rd0 = __uint_as_float((unsigned)b0);
  B.rd1 = __uint_as_float((unsigned)b1s);
  QMARK(4);
}

// rows: LDS buffer (>= 1 KiB, reused for the per-obstacle records) holding env A's obstacle row
// (planes x, y, r of stride os) at rows[0] and env B's at rows[3 os].  Per lane: its env's pose
// (px, py), ray-0 direction (c0r, s0r) and obstacle count nl (0: no env in this half).
__device__ __forceinline__ void lidar_wave2(float* rows, int os, int nl, float px, float py, float c0r,
                                            float s0r, const float2* rayoff, unsigned long long* slot,
                                            int* mark, int* mark2, Scan<float>& A, Scan<float>& B,
                                            QProf* qp = nullptr, int rotA = 0, int rotB = 0, int* wout = nullptr) {
  const int l = lane_id();
  const int jl = l & 31;
  const bool valid = jl < nl;
  const float* rb = rows + (l >= 32 ? 3 * os : 0);
  // read unconditionally: lanes past their env's obstacles (or of an absent env B) get slot padding
  // or stale LDS, and every use below is masked by `valid`
  const float ox = rb[jl], oy = rb[os + jl], rr = rb[2 * os + jl];
  const float dx = ox - px, dy = oy - py;
  const float d = l_sqrt(m_fma(dx, dx, dy * dy));
  const float key = valid ? d - rr : big<float>();                              // simple_env.py:205-206
  // ballots of plain compares ANDed on the SALU (a ballot of an ANDed condition makes the compiler
  // materialise it per lane first)
  const unsigned long long vm = ballot(valid);
  const unsigned long long tb = vm & ballot(key < (float)kTermDist);            // :334
  A.term = (unsigned)tb != 0u; B.term = (unsigned)(tb >> 32) != 0u;
  A.far = B.far = false;
  const bool far = (vm & ballot(d >= (float)(0.99 * kSensorMax))) != 0;
  lidar_window2(dx, dy, key, d, rr, valid, far, c0r, s0r, reinterpret_cast<float4*>(rows), WinLds{slot, mark, rayoff},
                mark2, A, B, qp, rotA, rotB, wout);
}

// Angular-window lidar for the f64 build (one env per wave).  The ray windows are sized in float from
// the f64 geometry (the 0.05-ray margin dwarfs the float rounding of the inputs), and every
// (obstacle, ray) pair in a window runs lidar_brute's exact f64 test on the same ray-0-frame operands
// (a, b, r^2 and the ray table), so the hits are brute's.  The winner per ray is the smallest key:
// ds_min_u64 on the order-preserving key bits with the low 6 bits replaced by the obstacle lane, i.e.
// keys equal to within 64 ulps resolve to the lower lane (brute: exact ties only; the reference's own
// tie order is unspecified).  The winner's reading is then recomputed exactly as lidar_brute does
// (reading_of), so readings are bit-identical to the brute loop.
struct WinLdsD {
  unsigned long long* slot;   // [128] per wave, armed with kSlotArm between envs
  int* mark;                  // [64]  per wave
  const double2* rayoff;      // [128] block-shared ray offset table (f64)
};
__device__ __forceinline__ unsigned long long ord_key64(double k) {   // double -> order-preserving u64
  const unsigned long long b = (unsigned long long)__double_as_longlong(k);
  return (b >> 63) ? ~b : (b | (1ull << 63));
}
template <bool RANGE_CHECK>
__device__ __forceinline__ void lidar_window_d(double dx, double dy, double key, double d, double rr, bool valid,
                                               double sp, double cp, const WinLdsD& L, Scan<double>& out) {
  const int l = lane_id();
  double a, b;
  to_ray0(dx, dy, ray_c(cp, sp, double(kStartC), double(kStartS)), ray_s(cp, sp, double(kStartC), double(kStartS)), a, b);
  const double r2 = rr * rr;
  const float inv = (float)(1.0 / kRes);
  float pr = fast_atan2((float)b, (float)a) * inv;    // as lidar_window2: branch cut in the blind sector
  pr = pr < -32.5f ? pr + 192.0f : pr;
  const float margin = (float)(kWinMargin * kRes);
  const float x = fminf((float)rr * __builtin_amdgcn_rcpf((float)d), 1.0f);
  const float hr = (fmaf((float)(kPi / 2 - 1) * x, x * x, x) + margin) * inv;
  const bool wide = (d <= rr * 1.001) | (hr >= 32.5f);
  const int lo = wide ? 0 : max(0, (int)ceilf(pr - hr));
  const int hi = wide ? 127 : min(127, (int)floorf(pr + hr));
  const int cnt = valid ? max(0, hi - lo + 1) : 0;
  const int incl = wave_incl_scan(cnt);
  const int off = wave_excl_of(incl);
  const int W = __builtin_amdgcn_readlane(incl, 63);
  const int mk0 = ((l + 1) << 16) | (lo - off + 32768);
  const unsigned long long kq = (ord_key64(key) & ~63ull) | (unsigned long long)l;
  const unsigned kq_lo = (unsigned)kq, kq_hi = (unsigned)(kq >> 32);
  int carry = 0;
  for (int base = 0; base < W; base += kWave) {       // wave-uniform pass count
    L.mark[l] = 0;                                    // (callers' LDS need not be cleared)
    if (cnt > 0 && off >= base && off < base + kWave) L.mark[off - base] = mk0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const int mk = max(wave_incl_max_asm(L.mark[l]), carry);
    carry = __builtin_amdgcn_readlane(mk, 63);
    const int q = base + l;
    const int jj = max((mk >> 16) - 1, 0);
    const int si = (q + (mk & 0xffff) - 32768) & 127;
    const double ja = __shfl(a, jj, kWave), jb = __shfl(b, jj, kWave), jr2 = __shfl(r2, jj, kWave);
    const unsigned long long jk = ((unsigned long long)(unsigned)__shfl((int)kq_hi, jj, kWave) << 32) |
                                  (unsigned)__shfl((int)kq_lo, jj, kWave);
    const double2 cs = L.rayoff[si];
    const double proj = m_fma(ja, cs.x, jb * cs.y);    // ray_pair's arithmetic
    const double perp = m_fma(ja, cs.y, -(jb * cs.x));
    const double delta = m_fma(-perp, perp, jr2);
    bool hit = (q < W) & (proj >= 0.0) & (delta >= 0.0);
    if (RANGE_CHECK) hit = hit && (proj - l_sqrt(delta)) < double(kSensorMax);   // :458
    if (hit) atomicMin(&L.slot[si], jk);
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const unsigned long long v0 = L.slot[l], v1 = L.slot[l + 64];
  L.slot[l] = kSlotArm;
  L.slot[l + 64] = kSlotArm;
  L.mark[l] = 0;
  const int bj0 = v0 == kSlotArm ? -1 : (int)(v0 & 63), bj1 = v1 == kSlotArm ? -1 : (int)(v1 & 63);
  const double2 t0 = L.rayoff[l], t1 = L.rayoff[l + 64];
  out.rd0 = reading_of(t0.x, t0.y, bj0, a, b, r2);
  out.rd1 = reading_of(t1.x, t1.y, bj1, a, b, r2);
}

// Two envs per wave for the f64 window lidar (<= 32 obstacles each), lidar_window_d's arithmetic with
// lidar_window2's layout: lanes 0..31 hold env A's obstacles, lanes 32..63 env B's, each lane in the
// ray-0 frame of its own env's pose; both envs' (obstacle, ray) pairs go into one expanded list whose
// slots are env A's rays then env B's [256].  The winner payload's low 6 bits are the obstacle lane
// (0..63, so it names the env too), and each reading is recomputed from the winner's (a, b, r^2) as
// lidar_brute does: readings bit-identical to lidar_window_d and to the brute loop.
__device__ __forceinline__ void lidar_wave2_d(const double* rows, int os, int nl, double px, double py, double sp,
                                              double cp, const double2* rayoff, unsigned long long* slot,
                                              int* mark, double4* rec, Scan<double>& A, Scan<double>& B) {
  const int l = lane_id();
  const int jl = l & 31;
  const bool valid = jl < nl;
  const double* rb = rows + (l >= 32 ? 3 * os : 0);
  // read unconditionally (lanes past their env's obstacles get padding; every use is masked by valid)
  const double ox = rb[jl], oy = rb[os + jl], rr = rb[2 * os + jl];
  const double dx = ox - px, dy = oy - py;
  const double d = l_sqrt(m_fma(dx, dx, dy * dy));
  const double key = valid ? d - rr : big<double>();                          // simple_env.py:205-206
  const unsigned long long vm = ballot(valid);
  const unsigned long long tb = vm & ballot(key < kTermDist);                  // :334
  A.term = (unsigned)tb != 0u; B.term = (unsigned)(tb >> 32) != 0u;
  A.far = B.far = false;
  const bool far = (vm & ballot(d >= 0.99 * kSensorMax)) != 0;               // :458 matters
  double a, b;
  to_ray0(dx, dy, ray_c(cp, sp, double(kStartC), double(kStartS)), ray_s(cp, sp, double(kStartC), double(kStartS)), a, b);
  const double r2 = rr * rr;
  const float inv = (float)(1.0 / kRes);
  float pr = fast_atan2((float)b, (float)a) * inv;    // branch cut in the blind sector (lidar_window2)
  pr = pr < -32.5f ? pr + 192.0f : pr;
  const float margin = (float)(kWinMargin * kRes);
  const float x = fminf((float)rr * __builtin_amdgcn_rcpf((float)d), 1.0f);
  const float hr = (fmaf((float)(kPi / 2 - 1) * x, x * x, x) + margin) * inv;
  const bool wide = (d <= rr * 1.001) | (hr >= 32.5f);
  const int lo = wide ? 0 : max(0, (int)ceilf(pr - hr));
  const int hi = wide ? 127 : min(127, (int)floorf(pr + hr));
  const int cnt = valid ? max(0, hi - lo + 1) : 0;
  const int incl = wave_incl_scan(cnt);
  const int off = wave_excl_of(incl);
  const int W = __builtin_amdgcn_readlane(incl, 63);
  // mark: owner lane + 1 in the high bits, slot offset (env B: + 128) in the low bits
  const int mk0 = ((l + 1) << 16) | (lo - off + (l >= 32 ? 128 : 0) + 32768);
  const unsigned long long kq = (ord_key64(key) & ~63ull) | (unsigned long long)l;
  // per-obstacle record as two 16-B planes (a, b) [64] and (r^2, key | lane) [64]: lane l's halves at a
  // 16-B stride, so the stores and the owners' gathers are bank-conflict free (a 32-B record stride
  // put lanes 4 apart on the same banks; round 5)
  double2* const recA = reinterpret_cast<double2*>(rec);
  double2* const recB = recA + kWave;
  recA[l] = make_double2(a, b);
  recB[l] = make_double2(r2, __longlong_as_double((long long)kq));
  const int mpass = cnt > 0 ? off >> 6 : -1;
  int carry = 0;
  for (int base = 0, pass = 0; base < W; base += kWave, ++pass) {   // wave-uniform pass count
    if (mpass == pass) mark[off & (kWave - 1)] = mk0;   // marks of earlier passes are <= carry
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const int mk = max(wave_incl_max_asm(mark[l]), carry);
    carry = __builtin_amdgcn_readlane(mk, 63);
    const int q = base + l;
    const int jj = max((mk >> 16) - 1, 0);
    const int si = (q + (mk & 0xffff) - 32768) & 255;
    const double2 oa = recA[jj], ob = recB[jj];
    const double4 o = make_double4(oa.x, oa.y, ob.x, ob.y);   // owner's (a, b, r^2, key | lane)
    const unsigned long long jk = (unsigned long long)__double_as_longlong(o.w);
    const double2 cs = rayoff[si & 127];
    const double proj = m_fma(o.x, cs.x, o.y * cs.y);  // ray_pair's arithmetic
    const double perp = m_fma(o.x, cs.y, -(o.y * cs.x));
    const double delta = m_fma(-perp, perp, o.z);
    bool hit = (q < W) & (proj >= 0.0) & (delta >= 0.0);
    if (far) hit = hit && (proj - l_sqrt(delta)) < double(kSensorMax);       // :458 (wave-uniform)
    if (hit) atomicMin(&slot[si], jk);
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const unsigned long long v0 = slot[l], v1 = slot[l + 64], v2 = slot[128 + l], v3 = slot[192 + l];
  slot[l] = kSlotArm; slot[l + 64] = kSlotArm; slot[128 + l] = kSlotArm; slot[192 + l] = kSlotArm;
  mark[l] = 0;
  // reading of the winner (reading_of's arithmetic, the winner's record from LDS)
  auto reading = [&](double c, double sn, unsigned long long v) {
    const double2 wa = recA[(int)(v & 63)], wb = recB[(int)(v & 63)];
    const double4 w = make_double4(wa.x, wa.y, wb.x, wb.y);
    const double proj = m_fma(w.x, c, w.y * sn);
    const double perp = m_fma(w.x, sn, -(w.y * c));
    const double delta = m_fma(-perp, perp, w.z);
    return v != kSlotArm ? proj - l_sqrt(delta) : double(kSensorMax);     // :457-459
  };
  const double2 t0 = rayoff[l], t1 = rayoff[l + 64];
  A.rd0 = reading(t0.x, t0.y, v0);
  A.rd1 = reading(t1.x, t1.y, v1);
  B.rd0 = reading(t0.x, t0.y, v2);
  B.rd1 = reading(t1.x, t1.y, v3);
  // the records are read by every lane above before the caller's next writes to this buffer (the
  // wave's LDS instructions complete in order)
}

template <typename R, int LID, typename Row>
__device__ __forceinline__ void lidar_wave(const Row& E, int n, R px, R py, R sp, R cp,
                                           const typename Vec2<R>::T* rayoff, unsigned long long* slot,
                                           int* mark, Scan<R>& out) {
  const int l = lane_id();
  const bool valid = l < n;
  R ox = R(0), oy = R(0), rr = R(0);
  if (valid) E.get(l, ox, oy, rr);
  const R dx = ox - px, dy = oy - py, r2 = rr * rr;
  const R d = l_sqrt(m_fma(dx, dx, dy * dy));
  const R key = valid ? d - rr : big<R>();                                      // simple_env.py:205-206
  out.term = ballot(valid & (key < R(kTermDist))) != 0;                       // :334
  out.far = ballot(valid & (d >= R(0.99 * kSensorMax))) != 0;
  if constexpr (std::is_same<R, float>::value && (LID & kLidWindow) != 0) {
    const WinLds W{slot, mark, rayoff};
    if (!out.far) lidar_window<false>(dx, dy, key, d, rr, valid, px, py, sp, cp, W, E, out);
    else lidar_window<true>(dx, dy, key, d, rr, valid, px, py, sp, cp, W, E, out);
    return;
  }
  if constexpr (std::is_same<R, double>::value && (LID & kLidWindow) != 0) {
    const WinLdsD W{slot, mark, rayoff};
    if (!out.far) lidar_window_d<false>(dx, dy, key, d, rr, valid, sp, cp, W, out);
    else lidar_window_d<true>(dx, dy, key, d, rr, valid, sp, cp, W, out);
    return;
  }
  const auto t0 = rayoff[l], t1 = rayoff[l + 64];
  lidar_brute<R, LID & (kLidSkip | kLidUnroll2)>(dx, dy, r2, key, d, rr, valid, n, out.far, sp, cp,
                                                  t0.x, t0.y, t1.x, t1.y, out);
}

// Reset-kernel LDS carve (16-B aligned pieces):
//   [ray offset table 128 x Vec2][pair slots 4 waves x 128 x u64][owner marks 4 x 64 x i32]
//   [one obstacle row per wave: x[64], y[64], r[64]]
template <typename R> __host__ __device__ constexpr size_t lds_rayoff_bytes() { return 128 * 2 * sizeof(R); }
constexpr size_t kLdsSlotBytes = (size_t)kWaves * 128 * 8;
constexpr size_t kLdsMarkBytes = (size_t)kWaves * 64 * 4;
template <typename R> __host__ __device__ constexpr size_t lds_head_bytes() {
  return lds_rayoff_bytes<R>() + kLdsSlotBytes + kLdsMarkBytes;
}

// Block prologue shared by the step and reset kernels: ray-offset table and slot init.
template <typename R>
__device__ __forceinline__ void lds_prologue(const State<R>& S, char* lds, int tid) {
  auto* rayoff = reinterpret_cast<typename Vec2<R>::T*>(lds);
  auto* slots = reinterpret_cast<unsigned long long*>(lds + lds_rayoff_bytes<R>());
  if (tid < kSensors) rayoff[tid] = typename Vec2<R>::T{S.ray_tab[2 * tid], S.ray_tab[2 * tid + 1]};
  for (int i = tid; i < kWaves * 128; i += kBlock) slots[i] = kSlotArm;
}

// --------------------------------------------------------------------------- wave-per-env scan
// Shared by the two fast step kernels (step_kernel_wave: dynamics + scan in one launch;
// dyn_kernel + scan_kernel: split).  Each wave owns EPW consecutive envs and, after one block
// barrier that publishes the ray table, shares nothing with the other waves of its block: the
// wave-per-env lidar loop keeps the NEXT envs' obstacle rows in flight (LDS-DMA) while the
// current ones are scanned; on the f32 window path two envs share each iteration.
//
// LDS: [ray table 128 x Vec2, block-shared]
//      [per wave: pair slots 256 x u64 | owner marks 64 x i32 | row buffers 2 x (2 rows, >= 1 KiB)]
__host__ __device__ constexpr size_t align16(size_t b) { return (b + 15) & ~(size_t)15; }
__host__ __device__ constexpr int obst_stride(int cap) { return (cap + 3) & ~3; }
template <typename R> __host__ __device__ constexpr int row_bytes(int cap) { return 3 * obst_stride(cap) * (int)sizeof(R); }
template <typename R> __host__ __device__ constexpr size_t wave_tab_bytes() { return kSensors * 2 * sizeof(R); }
// two rows, and at least the 64 per-obstacle records (a, b, r^2, key) lidar_window2 / lidar_wave2_d leave in it
template <typename R> __host__ __device__ constexpr size_t scan_rowbuf_bytes(int cap) {
  return align16(std::max((size_t)2 * row_bytes<R>(cap), (size_t)64 * 4 * sizeof(R)));
}
// lidar_wave2 keeps pass-1 owner marks (64 ints) in the tail of the row buffer the next two-env DMA
// fills (cap <= 32: two rows), in the wave-scan slices and in the block queue's 1 KiB row buffers
static_assert(2 * row_bytes<float>(32) + 64 * 4 <= (int)scan_rowbuf_bytes<float>(32), "f32 mark2 tail");
static_assert(2 * row_bytes<float>(32) + 64 * 4 <= 1024, "block-queue mark2 tail");
template <typename R> __host__ __device__ constexpr size_t lds_scan_slice(int cap) {
  return 256 * 8 + 64 * 4 + 2 * scan_rowbuf_bytes<R>(cap);
}
template <typename R> __host__ __device__ size_t lds_scan_bytes(int cap, int waves = kWaves) {
  return wave_tab_bytes<R>() + waves * lds_scan_slice<R>(cap);
}

// LDS-DMA copy of `bytes` (multiple of 16, <= 2 KiB) from global `src` into the wave-uniform
// LDS buffer `dst`: lane l moves 16-B piece l (and l + 64).  Inline asm so hipcc does not
// track it: the compiler would otherwise drain it with vmcnt(0) at the first LDS read it
// cannot prove disjoint, i.e. inside the scan it is meant to overlap.  Completion is counted
// by hand (vm_wait) before the buffer is read.
__device__ __forceinline__ void dma_copy(const void* src, void* dst, int bytes) {
  const int nchunk = bytes / 16;
  const char* g = reinterpret_cast<const char*>(src);
  const unsigned d = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)dst);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = i * kWave + lane_id();
    if (c < nchunk) {
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                   "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(g + 16 * (size_t)c), "s"(d + 16u * i * kWave) : "memory");
    }
  }
}
// Wait until at most N vector-memory operations are outstanding (gfx9 vmcnt counts loads,
// LDS-DMA and stores in issue order): everything older than the last N has completed.
// Hand-counted vmcnt waits around the untracked inline-asm LDS-DMA.  The USV_SAFE_VMCNT build
// (libusvhip_safe.so) turns every one into vmcnt(0); tests/test_gpu_r2.py checks it is bitwise
// identical to the product build, so a miscounted wait (a DMA still in flight when its rows are
// read) would show as a difference.
template <int N> __device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 16, "vmcnt field");
#ifdef USV_SAFE_VMCNT
  __builtin_amdgcn_s_waitcnt(0x0F70);         // vmcnt(0)
#else
  __builtin_amdgcn_s_waitcnt(0x0F70 | N);     // expcnt 7, lgkmcnt 15: no wait on those
#endif
}

template <typename R> struct ScanLds {
  typename Vec2<R>::T* rayoff;
  unsigned long long* slot;
  int* mark;
  R* row0;
  R* row1;
};
template <typename R>
__device__ __forceinline__ ScanLds<R> scan_lds(char* lds, int wave, int cap) {
  char* w = lds + wave_tab_bytes<R>() + wave * lds_scan_slice<R>(cap);
  R* r0 = reinterpret_cast<R*>(w + 256 * 8 + 64 * 4);
  return ScanLds<R>{reinterpret_cast<typename Vec2<R>::T*>(lds), reinterpret_cast<unsigned long long*>(w),
                    reinterpret_cast<int*>(w + 256 * 8), r0,
                    reinterpret_cast<R*>(reinterpret_cast<char*>(r0) + scan_rowbuf_bytes<R>(cap))};
}
// envs per scan iteration: two on the f32 window path (<= 32 obstacle lanes per env)
template <typename R, int LID> __device__ __forceinline__ int scan_step(int cap) {
  return ((LID & kLidWindow) != 0 && cap <= 32) ? 2 : 1;     // lidar_wave2 / lidar_wave2_d
}
// Issue the prologue DMAs (ray table by wave 0, the first iteration's rows) and arm the slots.
template <typename R, int LID>
__device__ __forceinline__ void scan_prologue(const State<R>& S, const ScanLds<R>& L, int wave, int e0, int ne) {
  const int cap = S.cap;
  if (wave == 0) dma_copy(S.ray_tab, L.rayoff, (int)wave_tab_bytes<R>());
  if (ne > 0) dma_copy(S.orow(e0), L.row0, min(scan_step<R, LID>(cap), ne) * row_bytes<R>(cap));
#pragma unroll
  for (int i = 0; i < 4; ++i) L.slot[i * 64 + lane_id()] = kSlotArm;
  L.mark[lane_id()] = 0;                              // lidar_window2 clears them after each call
}

// VALU issue is arbitrated by priority, then age (MI355X_MICROARCH.md, Two waves per SIMD): with
// a static split the oldest waves of a SIMD finish first and the youngest run alone at the end.
// The scan loops lower a wave's priority as it progresses (3 at the start, 0 in its last
// quarter), so the waves of a SIMD advance together and finish together.
__device__ __forceinline__ void set_prio(int p) {   // p wave-uniform
  if (p >= 3) __builtin_amdgcn_s_setprio(3);
  else if (p == 2) __builtin_amdgcn_s_setprio(2);
  else if (p == 1) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
}

// Outputs of one scanned env e (wave-wide, lane l holds rays l and l + 64): the sensor half of
// its obs row; for a done env the terminal obs and the stale scan; term / collision bit k.
template <typename R, int MODE>
__device__ __forceinline__ void emit_env(const State<R>& S, const IO<R>& io, int e, const Scan<R>& sc,
                                         unsigned trunc_bit, int k, unsigned& term_m, unsigned& coll_m) {
  const int l = lane_id();
  const bool done = sc.term || trunc_bit;
  const bool coll = ballot((sc.rd0 < R(kCollDist)) | (sc.rd1 < R(kCollDist))) != 0;  // :153-156
  term_m |= (unsigned)sc.term << k;
  coll_m |= (unsigned)coll << k;
  const float s0 = (float)l_norm(sc.rd0), s1 = (float)l_norm(sc.rd1);        // :82-83
  float* row = io.obs + (size_t)e * kObsDim;
  st_out(row + kHdr + l, s0);                                  // stale scan is kept by reset
  st_out(row + kHdr + 64 + l, s1);
  if (done) {
    if (io.fobs) {                                             // terminal obs
      float* f = io.fobs + (size_t)e * kObsDim;
      f[kHdr + l] = s0;
      f[kHdr + 64 + l] = s1;
      // header: written earlier by this wave (wave kernel), by dyn_kernel, or by wave 0 of this
      // block (kind 3, released before the block barrier)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      if (l < kHdr) f[l] = row[l];
    }
    if (S.autoreset == USV_AUTORESET_SAME_STEP) {
      S.sensor_last[(size_t)e * kSensors + l] = sc.rd0;
      S.sensor_last[(size_t)e * kSensors + 64 + l] = sc.rd1;
    }
  }
}

// The scan loop over this wave's ne envs.  Inputs lane-per-env (lane k = env e0 + k): pose
// P = (x, y, sin psi, cos psi), obstacle count nl, truncation bits trunc_m.  Writes the sensor
// half of each obs row, final obs and stale scan of done envs; returns term / collision bits.
// Precondition: the prologue DMAs have landed and the ray table is published.
template <typename R, int MODE, int LID>
__device__ __forceinline__ void scan_envs(const State<R>& S, const IO<R>& io, const ScanLds<R>& L, int e0,
                                          int ne, const R4<R>& P, int nl, unsigned trunc_m,
                                          unsigned& term_m, unsigned& coll_m, Prof& prof) {
  const int cap = S.cap;
  const int rowb = row_bytes<R>(cap);
  const int step = scan_step<R, LID>(cap);
  term_m = 0; coll_m = 0;
  auto emit = [&](int k, const Scan<R>& sc) {               // outputs of env e0 + k
    emit_env<R, MODE>(S, io, e0 + k, sc, (trunc_m >> k) & 1, k, term_m, coll_m);
  };
  const int iters = (ne + step - 1) / step;
  for (int k = 0; k < ne; k += step) {
    R* cur = ((k / step) & 1) ? L.row1 : L.row0;
    if (S.prio == 1) set_prio(3 - (4 * (k / step)) / iters);
    else if (S.prio == 2) set_prio(k + step >= ne ? 3 : 0);   // a wave's last iteration first
    prof.mark(4);
    // rows of this iteration landed: every env of the previous iteration issued its two
    // sensor-row stores after their DMA (a full pair: four), so all older ops are done
    if (k > 0) {
      if (step == 2) vm_wait<4>(); else vm_wait<2>();
    }
    if (k + step < ne)
      dma_copy(S.orow(e0 + k + step), ((k / step) & 1) ? L.row0 : L.row1, min(step, ne - k - step) * rowb);
    prof.mark(1);
    prof.count(7);
    if constexpr (std::is_same<R, float>::value && (LID & kLidWindow) != 0) {
      if (step == 2) {
        const bool hasB = k + 1 < ne;
        const bool hb = lane_id() >= 32;
        const int kl = hb ? k + 1 : k;             // this lane's env (B half: k + 1 if it exists)
        const int kc = hasB ? kl : k;
        const float lpx = __shfl(P.x, kc, kWave), lpy = __shfl(P.y, kc, kWave);
        const float lsp = __shfl(P.z, kc, kWave), lcp = __shfl(P.w, kc, kWave);
        const int lnl = (hb && !hasB) ? 0 : __shfl(nl, kc, kWave);
        Scan<float> sa, sb;
        // (pass-1 marks: the tail of the other row buffer, past the <= 768 B the next DMA fills)
        float* const oth = ((k / step) & 1) ? L.row0 : L.row1;
        lidar_wave2(cur, obst_stride(cap), lnl, lpx, lpy, ray_c(lcp, lsp, (float)kStartC, (float)kStartS),
                    ray_s(lcp, lsp, (float)kStartC, (float)kStartS), L.rayoff, L.slot, L.mark,
                    reinterpret_cast<int*>(oth) + 192, sa, sb);
        prof.mark(2);
        emit(k, sa);
        if (hasB) emit(k + 1, sb);
        prof.mark(3);
        continue;
      }
    }
    if constexpr (std::is_same<R, double>::value && (LID & kLidWindow) != 0) {
      if (step == 2) {                             // as above, f64 arithmetic (lidar_wave2_d)
        const bool hasB = k + 1 < ne;
        const bool hb = lane_id() >= 32;
        const int kl = hb ? k + 1 : k;
        const int kc = hasB ? kl : k;
        const double lpx = __shfl(P.x, kc, kWave), lpy = __shfl(P.y, kc, kWave);
        const double lsp = __shfl(P.z, kc, kWave), lcp = __shfl(P.w, kc, kWave);
        const int lnl = (hb && !hasB) ? 0 : __shfl(nl, kc, kWave);
        Scan<double> sa, sb;
        // the records overwrite this iteration's rows once every lane has read them (in-order LDS)
        lidar_wave2_d(cur, obst_stride(cap), lnl, lpx, lpy, lsp, lcp, L.rayoff, L.slot, L.mark,
                      reinterpret_cast<double4*>(cur), sa, sb);
        prof.mark(2);
        emit(k, sa);
        if (hasB) emit(k + 1, sb);
        prof.mark(3);
        continue;
      }
    }
    Scan<R> sc;
    const int os = obst_stride(cap);
    lidar_wave<R, LID>(RowSoA<R>{cur, cur + os, cur + 2 * os}, __builtin_amdgcn_readlane(nl, k), bcast(P.x, k),
                       bcast(P.y, k), bcast(P.z, k), bcast(P.w, k), L.rayoff, L.slot, L.mark, sc);
    prof.mark(2);
    emit(k, sc);
    prof.mark(3);
  }
}

// Epilogue shared by both: terminated flag and collision term of the reward (lane-per-env),
// then same-step autoreset of the done envs.
template <typename R, int MODE>
__device__ __forceinline__ void scan_epilogue(const State<R>& S, const IO<R>& io, int e0, int ne,
                                              R partial, bool have_partial, unsigned term_m,
                                              unsigned coll_m, unsigned trunc_m) {
  const int l = lane_id();
  if (l < ne) {
    const int e = e0 + l;
    const bool coll = (coll_m >> l) & 1;                                     // simple_env.py:153-156
    if (have_partial) st_out(io.rew + e, coll ? R(-20) + partial : partial);
    else if (coll) io.rew[e] = R(-20) + io.rew[e];
    io.term[e] = (term_m >> l) & 1;
    if (have_partial) io.trunc[e] = (trunc_m >> l) & 1;
    if (io.done) io.done[e] = ((term_m | trunc_m) >> l) & 1;
  }
  if (S.autoreset == USV_AUTORESET_SAME_STEP) {
    for (int k = 0; k < ne; ++k)
      if (((term_m | trunc_m) >> k) & 1) reset_wave<R, MODE>(S, e0 + k, io.obs + (size_t)(e0 + k) * kObsDim);
  }
}

// ---- fused: lane-per-env dynamics of the wave's own envs, then the scan
template <typename R, int MODE, int EPW, int LID>
__device__ __forceinline__ void step_body_wave(const State<R>& S, const IO<R>& io) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);   // wave-uniform (SGPR)
  const int l = lane_id();
  const int e0 = (blockIdx.x * kWaves + wave) * EPW;        // this wave's envs: e0 .. e0+ne-1
  const int ne = min(EPW, S.N - e0);
  const ScanLds<R> L = scan_lds<R>(lds, wave, S.cap);
  Prof prof;
  USV_STAMP_W(0);
  USV_STAMP_ID();
  if (S.prio == 1) __builtin_amdgcn_s_setprio(3);
  scan_prologue<R, LID>(S, L, wave, e0, ne);
  // dynamics: lanes 0..ne-1; lanes >= ne recompute env ne-1 and store identical values to the
  // identical addresses (benign) -- no divergent memory operations, so hipcc's own vmcnt
  // bookkeeping stays exact around the untracked DMAs
  R px = R(0), py = R(0), sp = R(0), cp = R(1);
  R partial = R(0);
  int nl = 0;
  bool trunc = false;
  if (ne > 0) {
    const int e = e0 + min(l, ne - 1);
    const float2 a = reinterpret_cast<const float2*>(io.act)[e];
    nl = S.I(I_NOBS)[e];                              // (ahead of the dynamics' stores)
    float hdr[kHdr];
    env_dynamics<R, MODE>(S, e, a.x, a.y, hdr, px, py, sp, cp, partial, trunc,
                             io.info ? io.info + (size_t)e * USV_INFO_DIM : nullptr);
    float* row = io.obs + (size_t)e * kObsDim;
#pragma unroll
    for (int i = 0; i < kHdr; ++i) row[i] = hdr[i];   // lane-per-env rows: plain stores (L2 merges them)
  }
  const unsigned trunc_m = (unsigned)ballot(trunc);
  USV_STAMP_W(1);
  // prologue DMAs landed (the dynamics' loads and stores were issued after them), then the
  // barrier publishes wave 0's ray table
  vm_wait<2>();
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (ne <= 0) return;
  USV_STAMP_W(2);
  prof.mark(0);
  unsigned term_m, coll_m;
  scan_envs<R, MODE, LID>(S, io, L, e0, ne, R4<R>{px, py, sp, cp}, nl, trunc_m, term_m, coll_m, prof);
  USV_STAMP_W(3);
  scan_epilogue<R, MODE>(S, io, e0, ne, partial, true, term_m, coll_m, trunc_m);
  prof.mark(5);
  prof.flush(blockIdx.x * kWaves + wave);
  USV_STAMP_W(6);
}

template <typename R, int MODE, int EPW, int LID>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_num_sgpr(80), amdgpu_num_vgpr(64)))
void step_kernel_wave_tight(State<R> S, IO<R> io) { step_body_wave<R, MODE, EPW, LID>(S, io); }

template <typename R, int MODE, int EPW, int LID>
__global__ __launch_bounds__(kBlock) void step_kernel_wave(State<R> S, IO<R> io) {
  step_body_wave<R, MODE, EPW, LID>(S, io);
}

// ---- split: dyn_kernel (full-width lane-per-env dynamics: state, obs header, partial reward
// into rew, truncation into trunc, pose record), then scan_kernel
template <typename R, int MODE>
__global__ __launch_bounds__(kBlock) void dyn_kernel(State<R> S, IO<R> io) {
  const int e = blockIdx.x * kBlock + threadIdx.x;
  if (e >= S.N) return;
  const float2 a = reinterpret_cast<const float2*>(io.act)[e];
  const int nob = S.I(I_NOBS)[e];                    // (ahead of the dynamics' stores)
  float hdr[kHdr];
  R px, py, sp, cp, partial;
  bool trunc;
  env_dynamics<R, MODE>(S, e, a.x, a.y, hdr, px, py, sp, cp, partial, trunc,
                             io.info ? io.info + (size_t)e * USV_INFO_DIM : nullptr);
  float* row = io.obs + (size_t)e * kObsDim;
#pragma unroll
  for (int i = 0; i < kHdr; ++i) row[i] = hdr[i];     // lane-per-env rows: plain stores (L2 merges them)
  S.pose[2 * (size_t)e] = R4<R>{px, py, sp, cp};
  S.pose[2 * (size_t)e + 1] = R4<R>{partial, R(nob), R(trunc ? 1 : 0), R(0)};
  io.rew[e] = partial;
  io.trunc[e] = trunc;
}

// WPB waves per block: 4 (256 threads) or 1 (64 threads: many small blocks, so the hardware
// dispatcher refills a SIMD as soon as one wave finishes and the drain tail is one small block)
template <typename R, int MODE, int EPW, int LID, int WPB>
__device__ __forceinline__ void scan_body(const State<R>& S, const IO<R>& io) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int wave = WPB == 1 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);   // SGPR
  const int l = lane_id();
  const int e0 = (blockIdx.x * WPB + wave) * EPW;
  const int ne = min(EPW, S.N - e0);
  const ScanLds<R> L = scan_lds<R>(lds, wave, S.cap);
  Prof prof;
  USV_STAMP_W(0);
  USV_STAMP_ID();
  scan_prologue<R, LID>(S, L, wave, e0, ne);
  // per-env inputs, lane-per-env (lanes >= ne repeat env ne-1), read once: the scan loop then
  // issues no vector loads and its counted vm_wait stays exact
  const int ec = max(0, min(e0 + min(l, ne - 1), S.N - 1));
  const R4<R> P = S.pose[2 * (size_t)ec];
  const int nl = S.I(I_NOBS)[ec];
  const unsigned trunc_m = (unsigned)ballot(io.trunc[ec] != 0);
  vm_wait<0>();
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (ne <= 0) return;
  USV_STAMP_W(1);
  prof.mark(0);
  unsigned term_m, coll_m;
  scan_envs<R, MODE, LID>(S, io, L, e0, ne, P, nl, trunc_m, term_m, coll_m, prof);
  USV_STAMP_W(3);
  scan_epilogue<R, MODE>(S, io, e0, ne, R(0), false, term_m, coll_m, trunc_m);
  prof.mark(5);
  prof.flush(blockIdx.x * WPB + wave);
  USV_STAMP_W(6);
}

template <typename R, int MODE, int EPW, int LID, int WPB>
__global__ __launch_bounds__(kWave * WPB) __attribute__((amdgpu_num_sgpr(80), amdgpu_num_vgpr(64)))
void scan_kernel_tight(State<R> S, IO<R> io) { scan_body<R, MODE, EPW, LID, WPB>(S, io); }

template <typename R, int MODE, int EPW, int LID, int WPB>
__global__ __launch_bounds__(kWave * WPB) void scan_kernel(State<R> S, IO<R> io) {
  scan_body<R, MODE, EPW, LID, WPB>(S, io);
}

// f64 scan compiled for more waves per SIMD (the uncapped f64 scan takes 141 VGPRs: 3 waves)
constexpr int kF64ScanWaves = 4;
template <typename R, int MODE, int EPW, int LID, int WPB>
__global__ __launch_bounds__(kWave * WPB) __attribute__((amdgpu_waves_per_eu(kF64ScanWaves, kF64ScanWaves)))
void scan_kernel_d(State<R> S, IO<R> io) { scan_body<R, MODE, EPW, LID, WPB>(S, io); }

// ---- fused with block-wide dynamics (kind 3, f64 usv-simple): wave 0 of each 4-wave block runs
// the dynamics of the block's 4 * EPW <= 64 envs lane-per-env (full width at EPW = 16, as the split
// dyn_kernel does) and hands each env's pose, obstacle count, partial reward and truncation to its
// scanning wave through LDS; waves 1..3 meanwhile wait at the barrier with their first rows in
// flight.  Same per-env arithmetic as kinds 1 and 2, one launch instead of two (no pose records
// through HBM, no second launch ramp).
template <typename R> __host__ __device__ constexpr size_t lds_blockdyn_bytes(int cap) {
  return (lds_scan_bytes<R>(cap) + 31) / 32 * 32 + 2 * kWave * sizeof(R4<R>);
}
template <typename R, int MODE, int EPW, int LID>
__device__ __forceinline__ void step_body_blockdyn(const State<R>& S, const IO<R>& io) {
  static_assert(kWaves * EPW <= kWave, "one dynamics lane per env of the block");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);   // wave-uniform (SGPR)
  const int l = lane_id();
  const int eb = blockIdx.x * kWaves * EPW;                 // the block's envs eb .. eb+nbe-1
  const int nbe = min(kWaves * EPW, S.N - eb);
  const int e0 = eb + wave * EPW;                           // this wave's envs e0 .. e0+ne-1
  const int ne = min(EPW, S.N - e0);
  const ScanLds<R> L = scan_lds<R>(lds, wave, S.cap);
  R4<R>* const rec = reinterpret_cast<R4<R>*>(lds + (lds_scan_bytes<R>(S.cap) + 31) / 32 * 32);
  Prof prof;
  USV_STAMP_W(0);
  USV_STAMP_ID();
  if (S.prio == 1) __builtin_amdgcn_s_setprio(3);
  scan_prologue<R, LID>(S, L, wave, e0, ne);
  if (wave == 0) {
    // lanes >= nbe recompute env nbe-1 and store identical values to identical addresses (no
    // divergent memory operations: hipcc's vmcnt bookkeeping stays exact around the DMAs)
    const int e = eb + min(l, nbe - 1);
    const float2 a = reinterpret_cast<const float2*>(io.act)[e];
    const int nob = S.I(I_NOBS)[e];                        // (ahead of the dynamics' stores)
    float hdr[kHdr];
    R px, py, sp, cp, partial;
    bool trunc;
    env_dynamics<R, MODE>(S, e, a.x, a.y, hdr, px, py, sp, cp, partial, trunc,
                          io.info ? io.info + (size_t)e * USV_INFO_DIM : nullptr);
    float* row = io.obs + (size_t)e * kObsDim;
#pragma unroll
    for (int i = 0; i < kHdr; ++i) row[i] = hdr[i];         // lane-per-env rows: plain stores
    rec[l] = R4<R>{px, py, sp, cp};
    rec[kWave + l] = R4<R>{partial, R(nob), R(trunc ? 1 : 0), R(0)};
    USV_STAMP_W(1);
    if (io.fobs || S.autoreset == USV_AUTORESET_SAME_STEP) {
      // waves 1-3 read these header rows back for their done envs' terminal obs (emit_env), and
      // reset their done envs, whose state this wave stored (same-step autoreset): every store
      // complete and released to the workgroup before the barrier, so no reset store of another
      // wave can be overtaken by one of these
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      vm_wait<0>();
    } else {
      vm_wait<2>();   // the prologue DMA landed: the header stores above were issued after it
    }
  } else {
    vm_wait<0>();
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // records + ray table published
  if (ne <= 0) return;
  USV_STAMP_W(2);
  prof.mark(0);
  const int k = wave * EPW + min(l, ne - 1);                // lane-per-env view of this wave's envs
  const R4<R> P = rec[k], M = rec[kWave + k];
  const unsigned trunc_m = (unsigned)ballot(M.z != R(0));
  unsigned term_m, coll_m;
  scan_envs<R, MODE, LID>(S, io, L, e0, ne, P, (int)M.y, trunc_m, term_m, coll_m, prof);
  USV_STAMP_W(3);
  scan_epilogue<R, MODE>(S, io, e0, ne, M.x, true, term_m, coll_m, trunc_m);
  prof.mark(5);
  prof.flush(blockIdx.x * kWaves + wave);
  USV_STAMP_W(6);
}

template <typename R, int MODE, int EPW, int LID>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kF64ScanWaves, kF64ScanWaves)))
void step_kernel_blockdyn(State<R> S, IO<R> io) { step_body_blockdyn<R, MODE, EPW, LID>(S, io); }

// ---- block-queue step (f32 window lidar, cap <= 32): 1024-thread blocks of 16 waves own
// kQE = 128 envs each; the block's env pairs are pulled from an LDS counter.  VALU issue on a
// SIMD is arbitrated by priority, then age, so with a static split the oldest waves finish first
// and the youngest run alone at the end; with the queue the favoured waves simply take more pairs
// and all of them finish together.
//   fused (usv-simple): waves 0 and 1 run the block's dynamics lane-per-env (full width) and
//                       leave one 64-B record per env in LDS;
//   split (usv-asmc-simple): dyn_rec_kernel ran first and left the records in S.qrec; they are
//                       DMA'd into LDS.
// Record (16 f32): pose (x, y, ray-0 direction c0, s0) | partial reward, n_obs | truncated << 16
// (int bits), then the non-constant obs-header values h0, h2..h9, h11 (make_header).  The obs
// header is stored together with the sensors when the env's pair is scanned, so each obs row is
// written once, late, and as a whole (no early header stores to lines that would be evicted
// before the sensors reach them).
// Each wave's first pair is static (pair = wave); its rows and the next pair's are DMA'd while
// the current pair is scanned (one DMA instruction per pair: two 384-B SoA rows).
// kQE = 128 envs on kQW = 16 waves per block-queue block, compiled for 8 waves per SIMD (kQWPE) in
// kQSgpr = 80 SGPRs
constexpr int kQSgpr = 80, kQWPE = 8;
// Issue priority in the block queue (round 5).  VALU issue on a SIMD goes by priority, then age, so a
// CU's older block (the first one dispatched to it) wins every tie against the younger one: in the
// round-4 timeline the older block ended at ~11.7 us and the younger ran alone, at 4 waves per SIMD,
// for its last ~6 us.  (1) The dynamics waves run phase 1 at priority 3 (the younger block's 14 other
// waves wait at its barrier for them while the older block scans), back to 0 after the barrier;
// (2) in a one-round grid (<= 2 blocks per CU) the second block of each CU (block index >= the CU
// count: blocks are dispatched one per CU first) raises kQYoungWaves of its 16 waves to priority 1,
// so the two blocks progress at more even rates.  Both only in a one-round grid (State::qyoung set):
// with more rounds (524 288 envs) the phase-1 priority cost 0.9 us of 161.  Same-box A/Bs (gpurun_out
// r5b-r5e): -0.27 to -0.67 us per launch at 65 536 envs (usv-simple), -0.95 us (usv-asmc-simple, whose
// q kernel has the same phase 1).
constexpr int kQPrioDyn = 3, kQYoungWaves = 10;
constexpr int kQW = 16, kQE = 128, kQRec = 16;
__host__ __device__ constexpr size_t q_slice_bytes() { return 256 * 8 + 64 * 4 + 2 * 1024; }

// One DMA instruction (<= 64 pieces of 16 B, i.e. <= 1 KiB): pieces c >= nchunk are not copied.
// src is wave-uniform: SGPR base + a 32-bit lane offset (the saddr form), so no per-lane 64-bit
// address is kept live across the pair loop.
__device__ __forceinline__ void dma_copy1(const void* src, void* dst, int bytes) {
  const int c = lane_id();
  const unsigned d = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)dst);
  const uint64_t a = (uint64_t)(uintptr_t)src;
  // (readfirstlane returns int: widen through unsigned, or the low half would sign-extend)
  const uint64_t sb = ((uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)(a >> 32)) << 32) |
                      (uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)a);
  if (c < bytes / 16) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(16 * c), "s"(sb), "s"(d) : "memory");
  }
}

// dma_copy1 from a loop-invariant wave-uniform base (SGPR pair) at a wave-uniform byte offset `off`
// carried in the lanes' 32-bit offsets: the pair loop then computes no 64-bit row address per pair.
__device__ __forceinline__ void dma_copy_at(const void* base, int off, void* dst, int bytes) {
  const int c = lane_id();
  const unsigned d = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)dst);
  const uint64_t a = (uint64_t)(uintptr_t)base;
  const uint64_t sb = ((uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)(a >> 32)) << 32) |
                      (uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)a);
  if (c < bytes / 16) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(16 * c + off), "s"(sb), "s"(d) : "memory");
  }
}

__device__ __forceinline__ void make_qrec(float* rec, float px, float py, float sp, float cp, float partial,
                                          int n, bool trunc, const float (&h)[kHdr]) {
  const float c0 = ray_c(cp, sp, (float)kStartC, (float)kStartS), s0 = ray_s(cp, sp, (float)kStartC, (float)kStartS);
  float4* r4 = reinterpret_cast<float4*>(rec);
  r4[0] = make_float4(px, py, c0, s0);
  r4[1] = make_float4(partial, __int_as_float(n | (trunc ? 1 << 16 : 0)), h[0], h[2]);
  r4[2] = make_float4(h[3], h[4], h[5], h[6]);
  r4[3] = make_float4(h[7], h[8], h[9], h[11]);
}
// obs-header value i (0..14) of the env whose record is `rec` (make_header's layout: entries 1, 10,
// 13 are 0, entries 12, 14 the max_acceleration constants)
__device__ __forceinline__ float qrec_hdr(const float* rec, int i) {
  const float v = rec[i == 0 ? 6 : (i <= 9 ? i + 5 : 15)];
  return (i == 1 || i == 10 || i == 13) ? 0.0f
       : i == 12 ? (float)(kMaxAccU / 10.0) : i == 14 ? (float)(kMaxAccR / 10.0) : v;
}

// Terminal obs and stale scan of a done env e (rare path; lane l holds its rays l, l + 64).
// `rot`: the scan is rotated across lanes (lane l holds rays (l - rot) & 63 and 64 + that).
__device__ __forceinline__ void q_emit_done(const State<float>& S, const IO<float>& io, int e,
                                            const Scan<float>& sc, const float* rec, int rot) {
  const int l = lane_id();
  const int ray = (l - rot) & (kWave - 1);
  if (io.fobs) {
    float* f = io.fobs + (size_t)e * kObsDim;
    f[kHdr + ray] = l_norm(sc.rd0);
    f[kHdr + 64 + ray] = l_norm(sc.rd1);
    const int hi = min(l, kHdr - 1);
    f[hi] = qrec_hdr(rec, hi);
  }
  if (S.autoreset == USV_AUTORESET_SAME_STEP) {
    S.sensor_last[(size_t)e * kSensors + ray] = sc.rd0;
    S.sensor_last[(size_t)e * kSensors + 64 + ray] = sc.rd1;
  }
}

// Two block shapes: QE = 128 envs on QW = 16 waves (the default, two blocks per CU), and QE = 16 envs
// on QW = 8 waves for small env counts, where 128-env blocks would leave most CUs idle (4 096 envs
// are 32 such blocks) -- each wave then owns about one pair, and up to four blocks share a CU.
constexpr int kQE_S = 16, kQW_S = 8;
constexpr int kQSmallBelow = 32768;   // env count below which the small blocks are the default (tools/nsweep.sh)
template <int QE = kQE, int QW = kQW> __host__ __device__ constexpr size_t lds_q_bytes() {
  return wave_tab_bytes<float>() + QW * q_slice_bytes() + QE * kQRec * 4 + 16 + QE * 4;   // + n_obs[QE]
}
static_assert(2 * lds_q_bytes() <= 160 * 1024, "two blocks per CU");
static_assert(4 * lds_q_bytes<kQE_S, kQW_S>() <= 160 * 1024, "four small blocks per CU");

// DONE: also write the done mask (io.done, ABI v4).  A template switch rather than a runtime test:
// the raw step (usv_step, io.done null) then carries neither the pointer nor its branch in the pair
// loop, whose SGPR budget is at its limit (a runtime test cost 0.25 us per launch).
// CHAIN = false (usv-asmc-simple, FUSED): asmc_chain_kernel ran the ASMC chain, phase 1 the rest.
// INFO (fused): phase 1 writes the per-step info rows (usv_step_ex with info_dev); a template switch
// like DONE: the info path's registers would otherwise make phase 1 spill, and the spill's reload
// wait for every store the dynamics issued before the barrier.
template <int MODE, bool FUSED, bool DONE = false, int kQE = ::usv::kQE, int kQW = ::usv::kQW, bool CHAIN = true,
          bool INFO = false, bool SPAN = false>
__device__ __forceinline__ void step_q_body(const State<float>& S, const IO<float>& io) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int l = lane_id();
  constexpr int os = 32, rowb = row_bytes<float>(32);  // cap in [29, 32]: plane stride 32, 384-B rows
  const int eb = blockIdx.x * kQE;                     // this block's envs: eb .. eb + nbe - 1
  const int nbe = min(kQE, S.N - eb);
  const int np = (nbe + 1) >> 1;                       // and pairs 0 .. np - 1 (block-local)
  char* const slice = lds + wave_tab_bytes<float>() + wave * q_slice_bytes();
  unsigned long long* const slot = reinterpret_cast<unsigned long long*>(slice);
  int* const mark = reinterpret_cast<int*>(slice + 256 * 8);
  float* const rowbuf0 = reinterpret_cast<float*>(slice + 256 * 8 + 64 * 4);
  float* const rowbuf1 = rowbuf0 + 256;
  float* const recs = reinterpret_cast<float*>(lds + wave_tab_bytes<float>() + kQW * q_slice_bytes());
  unsigned* const qctr = reinterpret_cast<unsigned*>(recs + kQE * kQRec);
  int* const qnob = reinterpret_cast<int*>(recs + kQE * kQRec) + 4;   // fused: the block's n_obs
  const float2* const rayoff = reinterpret_cast<const float2*>(lds);
#ifdef USV_DIAG_QPROF
  QProf qprof;
  QProf* const qp = &qprof;
#else
  QProf* const qp = nullptr;
#endif
  // qctr[1 + w]: dynamics wave w's state stores are acknowledged (set after the barrier, below; a
  // wave that same-step-resets one of wave w's envs waits for it, so its reset stores cannot be
  // overtaken by them)
  unsigned* const qdyn = qctr + 1;
  if (threadIdx.x == 0) {
    qctr[0] = kQW;                                     // pairs 0 .. kQW-1 are the static first ones
    qdyn[0] = 0u;
    qdyn[1] = 0u;
  }

  // the ray table: by the last wave, so that the dynamics waves (fused) issue no DMA of their own
  if (wave == kQW - 1) dma_copy(S.ray_tab, lds, (int)wave_tab_bytes<float>());
#pragma unroll
  for (int i = 0; i < 4; ++i) slot[i * 64 + l] = kSlotArm;
  mark[l] = 0;                                         // lidar_window2 clears them after each call
  USV_STAMP_W(0);
  USV_STAMP_ID();
  int cur = wave < np ? wave : -1;
  // first (static) pairs: pair w's rows into wave w's buffer 0.  With the fused dynamics, waves 2 and 3
  // also issue those of waves 0 and 1, whose state loads would otherwise queue behind their own DMA
  // (a wave's loads return in issue order); the barrier below publishes them.
  constexpr int kDynWaves = FUSED ? (kQE + kWave - 1) / kWave : 0;
  static_assert(kQW >= 3 * kDynWaves + 1 && 2 * kQW <= kQE + 2 * kWave, "block shape");
  // the store flags qdyn[0..kDynWaves-1] live in the 16-B qctr words (lds_q_bytes), before qnob
  static_assert(kDynWaves <= 2, "qdyn holds two dynamics waves' flags");
  if (wave >= kDynWaves && cur >= 0) dma_copy1(S.orow(eb + 2 * cur), rowbuf0, min(2, nbe - 2 * cur) * rowb);
  if (FUSED && wave >= kDynWaves && wave < 2 * kDynWaves) {
    const int w = wave - kDynWaves;
    if (w < np)
      dma_copy1(S.orow(eb + 2 * w), lds + wave_tab_bytes<float>() + w * q_slice_bytes() + 256 * 8 + 64 * 4,
                min(2, nbe - 2 * w) * rowb);
  }
  if constexpr (FUSED) {
    // the block's obstacle counts into LDS by waves 2 kDynWaves .. 3 kDynWaves - 1 (one env per lane),
    // so the dynamics waves load nothing after their stores: a load issued after them would make the
    // wave wait for every store's ack (one vmcnt counter) before the barrier
    if (wave >= 2 * kDynWaves && wave < 3 * kDynWaves) {
      const int k = (wave - 2 * kDynWaves) * kWave + l;
      if (k < nbe) qnob[k] = S.I(I_NOBS)[eb + k];
    }
    // dynamics, one lane per env.  Lanes past the end repeat the wave's last env (same wave:
    // every lane loads the state before any lane stores it); a wave with no env of its own must
    // not run, or two waves would race on the same env's state
    if (wave < kDynWaves && wave * kWave < nbe) {
      if (S.qyoung != INT_MAX) __builtin_amdgcn_s_setprio(kQPrioDyn);
      const int k = min(wave * kWave + l, nbe - 1);
      const int e = eb + k;
      const float2 a = reinterpret_cast<const float2*>(io.act)[e];
      float hdr[kHdr];
      float px, py, sp, cp, partial;
      bool trunc;
      env_dynamics<float, MODE, CHAIN>(S, e, a.x, a.y, hdr, px, py, sp, cp, partial, trunc,
                                       INFO ? io.info + (size_t)e * USV_INFO_DIM : nullptr);
      io.trunc[e] = trunc;
      make_qrec(recs + k * kQRec, px, py, sp, cp, partial, 0, trunc, hdr);   // (n_obs: qnob)
    }
  } else {
    if (wave < kQE / 16 && wave * 16 < nbe)            // 16 records (1 KiB) per wave
      dma_copy1(S.qrec + (size_t)(eb + wave * 16) * kQRec, recs + wave * 16 * kQRec, min(16, nbe - wave * 16) * kQRec * 4);
  }
  // rows, ray table and records landed (the dynamics waves issued no DMA: their stores drain later,
  // ahead of their first pair's rows in the vmcnt order)
  USV_STAMP_W(1);
  if (wave >= kDynWaves) vm_wait<0>();
  QMARK(10);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (FUSED && wave < kDynWaves) __builtin_amdgcn_s_setprio(0);
  if ((int)blockIdx.x >= S.qyoung && wave < kQYoungWaves) __builtin_amdgcn_s_setprio(1);
  // Same-step reset ordering: a dynamics wave stored its envs' state in phase 1, and
  // another wave may reset one of those envs later in this launch; two waves' stores to one address
  // are ordered only if the first is acknowledged before the second is issued.  So each dynamics
  // wave drains its stores here, after the barrier (its first pair's rows are already in LDS, and
  // env_dynamics issues the state stores as soon as the new state exists, so little is left to
  // wait for), and sets its flag; a reset of one of its envs waits for the flag.  Measured against
  // no ordering at all: +0.1 us at 65 536 envs, +0.15 us at 524 288 (a per-pair flag in the loop
  // cost 0.5 / 1.8 us, draining before the barrier 0.05 / 1.6 us; gpurun_out r5h, r5i).
  if (FUSED && wave < kDynWaves) {
    vm_wait<0>();
    __hip_atomic_store(qdyn + wave, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  USV_STAMP_W(2);
  QMARK(0);
  unsigned tk = 0;
  if (l == 0) tk = atomicAdd(qctr, 1u);                 // LDS ticket of this wave's second pair
  // same-step autoresets of a pair run outside the pair loop (the loop is left and re-entered):
  // inside it their registers would spill the loop's to scratch
  int it = 0;
#ifdef USV_DIAG_STAMPS
  unsigned wsum = 0;                                   // (diagnostic: window sizes of this wave's pairs)
#endif
  const bool hb = l >= 32;
  auto pair_hasb = [&](int p) { return 2 * p + 1 < nbe; };
  const float* const oblk = S.orow(eb);               // this block's obstacle rows (pair p at 2 p rowb bytes)

  // An env pair's two obs rows are one 1144-B span, stored as five 256-B wave stores from the span's
  // first 32-B sector: every sector but the two at the span's ends is written whole by one write-through
  // store (the four sensor halves and the header store of round 3 split ~3 sectors per row between
  // instructions, 1.18x the algorithmic write bytes).  sh = the span's dword offset in its sector.
  const unsigned ob = (unsigned)(((uintptr_t)io.obs >> 2) & 7);
  auto pair_shift = [&](int p) { return (int)((ob + (unsigned)(eb + 2 * p) * (unsigned)kObsDim) & 7u); };
  // per-row layout (SPAN = false): the obs-header lanes are loop-invariant, packed in one register:
  // lanes 0..14 store env A's header value hi, 15..29 env B's, 30..63 repeat lane 29; the record slot
  // of value hi (qrec_hdr) in bits 8..12, bit 16: env B's lane, bit 17: a constant entry (1, 10, 12-14)
  int hpk = 0;
  if constexpr (!SPAN) {
    const int hl = min(l, 2 * kHdr - 1);
    const int hi = hl >= kHdr ? hl - kHdr : hl;
    const int hrec = hi == 0 ? 6 : (hi <= 9 ? hi + 5 : 15);
    hpk = hi | (hrec << 8) | ((hl >= kHdr) << 16) | ((hi == 1 || hi == 10 || hi >= 12) << 17);
  }
  // env record of pair c for this lane (lanes 0..31 env A, 32..63 env B; env A again when there is
  // no B): pose, meta and the obs-header value this lane stores (lanes sh..sh+14: env A's entries
  // 0..14, sh+15..sh+29: env B's; no env B: sh = 0 and lanes 15..29 repeat env A's).  Read one pair
  // ahead (after the current pair's scan), so the LDS latency overlaps the current pair's stores.
  auto rec_of = [&](int c, float4& P, float4& M, float& H) {
    const int c0 = 2 * c;
    const bool cB = pair_hasb(c);
    const int kk = (hb && cB) ? c0 + 1 : c0;
    const float* const rk = recs + kk * kQRec;
    P = *reinterpret_cast<const float4*>(rk);
    M = *reinterpret_cast<const float4*>(rk + 4);
    if constexpr (FUSED) M.y = __int_as_float(__float_as_int(M.y) | qnob[kk]);   // n_obs | truncated << 16
    if constexpr (!SPAN) {                             // (the constant entries are selected at the store)
      H = recs[((((hpk >> 16) & 1) && cB) ? c0 + 1 : c0) * kQRec + ((hpk >> 8) & 31)];
      return;
    }
    const int hl = min(max(l - ((SPAN && cB) ? pair_shift(c) : 0), 0), 2 * kHdr - 1);
    const int hi = hl >= kHdr ? hl - kHdr : hl;
    float v = recs[((hl >= kHdr && cB) ? c0 + 1 : c0) * kQRec + (hi == 0 ? 6 : (hi <= 9 ? hi + 5 : 15))];
    // make_header's constant entries 1, 10, 13 (0) and 12, 14 (max_acceleration / 10), as selects:
    // written as one conditional chain the compiler branches on exec around the record read
    const bool cst = ((0x7402 >> hi) & 1) != 0;
    const float hc = hi == 12 ? (float)(kMaxAccU / 10.0) : (hi == 14 ? (float)(kMaxAccR / 10.0) : 0.0f);
    asm volatile("" : "+v"(v));
    H = cst ? hc : v;
  };
  for (;;) {
    unsigned done = 0;
    int de0 = 0;
    float4 pose = make_float4(0.f, 0.f, 0.f, 0.f), meta = pose;
    float hv = 0.0f;
    if (cur >= 0) rec_of(cur, pose, meta, hv);
    while (cur >= 0) {
      int nxt = (int)__builtin_amdgcn_readlane(tk, 0);
      QCOUNT(8, 1);
      const bool odd = (it & 1) != 0;
      float* const cbuf = odd ? rowbuf1 : rowbuf0;
      float* const nbuf = odd ? rowbuf0 : rowbuf1;
      const int k0 = 2 * cur;
      const int e0 = eb + k0;
      const bool hasB = pair_hasb(cur);
      if (nxt >= np) nxt = -1;
      if (nxt >= 0) {                                  // wave-uniform
        if (l == 0) tk = atomicAdd(qctr, 1u);
        dma_copy_at(oblk, 2 * rowb * nxt, nbuf, (pair_hasb(nxt) ? 2 : 1) * rowb);
      }
      // this lane's env: lanes 0..31 env A, 32..63 env B (env A again when there is no B)
      const int kl = (hb && hasB) ? k0 + 1 : k0;
      const int el = e0 + (kl - k0);
      const int nt = __float_as_int(meta.y);
      // the pair's span offset and the lane rotations of the two scans that put each reading in the
      // lane that stores it (no env B: the rows are stored as in round 3, unrotated)
      const bool span2 = SPAN && hasB;
      const int sh = span2 ? pair_shift(cur) : 0;
      const int rotA = span2 ? kHdr + sh : 0, rotB = span2 ? 2 * kHdr + sh : 0;
      Scan<float> sa, sb;
      QMARK(1);
#ifdef USV_DIAG_STAMPS
      int wq = 0;
      lidar_wave2(cbuf, os, (hb && !hasB) ? 0 : (nt & 0xffff), pose.x, pose.y, pose.z, pose.w, rayoff, slot,
                  mark, reinterpret_cast<int*>(nbuf) + 192, sa, sb, qp, rotA, rotB, &wq);
      wsum += (unsigned)wq;
#else
      lidar_wave2(cbuf, os, (hb && !hasB) ? 0 : (nt & 0xffff), pose.x, pose.y, pose.z, pose.w, rayoff, slot,
                  mark, reinterpret_cast<int*>(nbuf) + 192, sa, sb, qp, rotA, rotB);
#endif
      float4 pose_n = pose, meta_n = meta;
      float hv_n = hv;
      if (nxt >= 0) rec_of(nxt, pose_n, meta_n, hv_n);   // the next pair's record (wave-uniform)
      // collision (:153-156): two compares and ballots per env (a fminf of the two readings would
      // canonicalise both first)
      const float kc = (float)kCollDist;
      const bool collA = (ballot(sa.rd0 < kc) | ballot(sa.rd1 < kc)) != 0;
      const bool collB = hasB ? (ballot(sb.rd0 < kc) | ballot(sb.rd1 < kc)) != 0 : collA;
      const bool termB = hasB ? sb.term : sa.term;
      float* const rowA = io.obs + (size_t)e0 * kObsDim;
      // the obs rows (header :91-96, sensors :82-83): five stores either way, so the loop's count of
      // memory instructions stays static (vm_wait below)
      if (span2) {
        // span dword 64 j + l - sh = lane l of store j: [header A | sensors A | header B | sensors B]
        float* const span = rowA - sh;
        const float a0 = l_norm(sa.rd0), a1 = l_norm(sa.rd1), b0 = l_norm(sb.rd0), b1 = l_norm(sb.rd1);
        const bool mA = l < kHdr + sh, mB = l < 2 * kHdr + sh;
        if (l >= sh) st_obs(span + l, mA ? hv : a0);   // (lanes < sh: the previous pair's dwords)
        st_obs(span + 64 + l, mA ? a0 : a1);
        st_obs(span + 128 + l, mA ? a1 : (mB ? hv : b0));
        st_obs(span + 192 + l, mB ? b0 : b1);
        if (mB) st_obs(span + 256 + l, b1);             // (lanes >= 30 + sh: the next pair's)
      } else {
        // per-row pieces: each row's sensors in two 256-B stores and the two headers in one (a lone
        // env, odd env count: env A's row twice, identical values to identical addresses)
        {
        float* const rowB = rowA + (hasB ? kObsDim : 0);
        st_obs(rowA + kHdr + l, l_norm(sa.rd0));
        st_obs(rowA + kHdr + 64 + l, l_norm(sa.rd1));
        st_obs(rowB + kHdr + l, l_norm(hasB ? sb.rd0 : sa.rd0));
        st_obs(rowB + kHdr + 64 + l, l_norm(hasB ? sb.rd1 : sa.rd1));
        if constexpr (SPAN) {
          const int hl = min(l, 2 * kHdr - 1);         // lanes 0..14 env A, 15..29 env B (or A again)
          st_obs((hl >= kHdr ? rowB - kHdr : rowA) + hl, hv);
        } else {
          const int hi = hpk & 31;
          const bool hB = ((hpk >> 16) & 1) && hasB;    // (no env B: env A's value again)
          const float hc = hi == 12 ? (float)(kMaxAccU / 10.0) : hi == 14 ? (float)(kMaxAccR / 10.0) : 0.0f;
          st_obs(rowA + (hB ? kObsDim : 0) + hi, ((hpk >> 17) & 1) ? hc : hv);
        }
        }
      }
      const bool term_l = hb ? termB : sa.term;         // reward, terminated: lanes 0..31 env A,
      const bool coll_l = hb ? collB : collA;           // 32..63 env B
      st_out(io.rew + el, coll_l ? -20.0f + meta.x : meta.x);
      io.term[el] = term_l;
      const bool done_l = term_l | ((nt >> 16) & 1);
      if constexpr (DONE) io.done[el] = done_l;        // (>= 7 stores still follow the DMA)
      const unsigned long long dm = ballot(done_l);
      const bool doneA = (unsigned)dm != 0u, doneB = hasB && (unsigned)(dm >> 32) != 0u;
      if (doneA | doneB) {
        if (doneA) q_emit_done(S, io, e0, sa, recs + k0 * kQRec, rotA);
        if (doneB) q_emit_done(S, io, e0 + 1, sb, recs + (k0 + 1) * kQRec, rotB);
      }
      // the next pair's rows landed: at least seven stores (four sensor halves, the headers, the
      // rewards and the terminated flags) were issued after their DMA
      QMARK(5);
      vm_wait<7>();
      QMARK(6);
      if (it == 0) USV_STAMP_W(5);                      // (diagnostic: first pair done)
      cur = nxt;
      pose = pose_n;
      meta = meta_n;
      hv = hv_n;
      ++it;
      if (S.autoreset == USV_AUTORESET_SAME_STEP && (doneA | doneB)) {
        done = (doneA ? 1u : 0u) | (doneB ? 2u : 0u);
        de0 = e0;
        break;
      }
    }
    if (!done) break;
    QMARK(11);
    for (; done; done &= done - 1) {
      const int e = de0 + __builtin_ctz(done);
      if constexpr (FUSED) {
        // the env's phase-1 stores (by dynamics wave (e - eb) / 64) are acknowledged before its reset
        // stores are issued: two waves' stores to one address are otherwise unordered
        const unsigned* const f = qdyn + ((e - eb) >> 6);
        while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)
          __builtin_amdgcn_s_sleep(2);
      }
      reset_wave<float, MODE>(S, e, io.obs + (size_t)e * kObsDim);
    }
    QMARK(7);
  }
  QMARK(11);
  qprof_flush(qp);
#ifdef USV_DIAG_STAMPS
  USV_STAMP_V(4, (unsigned long long)it | ((unsigned long long)wsum << 16));   // (pairs | window sizes << 16)
#endif
  USV_STAMP_W(3);
  USV_STAMP_W(6);
}

template <int MODE, bool FUSED, bool DONE, bool CHAIN = true, bool INFO = false, bool SPAN = false>
__global__ __launch_bounds__(kQW * kWave) __attribute__((amdgpu_num_sgpr(kQSgpr), amdgpu_waves_per_eu(kQWPE, kQWPE)))
void step_q_kernel(State<float> S, IO<float> io) { step_q_body<MODE, FUSED, DONE, kQE, kQW, CHAIN, INFO, SPAN>(S, io); }
template <int MODE, bool DONE, bool CHAIN = true, bool INFO = false>
__global__ __launch_bounds__(kQW_S * kWave) __attribute__((amdgpu_num_sgpr(80), amdgpu_waves_per_eu(8, 8)))
void step_qs_kernel(State<float> S, IO<float> io) { step_q_body<MODE, true, DONE, kQE_S, kQW_S, CHAIN, INFO>(S, io); }

// Split block-queue step, first half: full-width lane-per-env dynamics writing the env records
// (make_qrec) for step_q_kernel<MODE, false, DONE>, plus truncated and the info row.
template <int MODE>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, 2))) void dyn_rec_kernel(State<float> S, IO<float> io) {
  const int e = blockIdx.x * kBlock + threadIdx.x;
  if (e >= S.N) return;
  const float2 a = reinterpret_cast<const float2*>(io.act)[e];
  const int nob = S.I(I_NOBS)[e];                  // (ahead of the dynamics' stores)
  float hdr[kHdr];
  float px, py, sp, cp, partial;
  bool trunc;
  env_dynamics<float, MODE>(S, e, a.x, a.y, hdr, px, py, sp, cp, partial, trunc,
                            io.info ? io.info + (size_t)e * USV_INFO_DIM : nullptr);
  io.trunc[e] = trunc;
  make_qrec(S.qrec + (size_t)e * kQRec, px, py, sp, cp, partial, nob, trunc, hdr);
}

// usv-asmc-simple, split at the ASMC chain (kind 6): the two UsvAsmc.compute calls of every env,
// lane per env, pose and velocity stored back; step_q_kernel<ASMC_SIMPLE, true, DONE, false> then runs
// UsvSimpleEnv.step(zeros(2)) on them in its fused phase 1.  The chain is a long dependent VALU
// stream (one wave per SIMD at 65 536 envs); this kernel holds nothing else, so it carries no records,
// headers or rewards, and the q kernel's phase 1 does that part at full width.
template <typename R>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, 2))) void asmc_chain_kernel(State<R> S, IO<R> io) {
  const int e = blockIdx.x * kBlock + threadIdx.x;
  if (e >= S.N) return;
  const float2 a = reinterpret_cast<const float2*>(io.act)[e];
  R x = S.F(F_X)[e], y = S.F(F_Y)[e], psi = S.F(F_PSI)[e];
  R u = S.F(F_U)[e], v = S.F(F_V)[e], r = S.F(F_R)[e];
  asmc_env_chain<R>(S, e, S.I(I_ELAPSED)[e], a.x, a.y, x, y, psi, u, v, r);
  S.F(F_X)[e] = x; S.F(F_Y)[e] = y; S.F(F_PSI)[e] = psi;
  S.F(F_U)[e] = u; S.F(F_V)[e] = v; S.F(F_R)[e] = r;
}

// --------------------------------------------------------------------------- reset kernel
// Explicit (host-requested) reset of masked envs.  Reset obs = new header + the stale
// sensor_data: the scan at the last stepped pose (recomputed when that pose is still the
// current one, else the stored one; zeros for a never-stepped env), simple_env.py:302.
template <typename R, int MODE>
__global__ __launch_bounds__(kBlock) void reset_kernel(State<R> S, IO<R> io) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  auto* rayoff = reinterpret_cast<typename Vec2<R>::T*>(lds);
  auto* slots = reinterpret_cast<unsigned long long*>(lds + lds_rayoff_bytes<R>());
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);   // wave-uniform (SGPR)
  const int l = lane_id();
  const int e0 = blockIdx.x * kEPBReset;
  const int ne = S.N - e0 < kEPBReset ? S.N - e0 : kEPBReset;
  int* marks = reinterpret_cast<int*>(lds + lds_rayoff_bytes<R>() + kLdsSlotBytes);
  // one obstacle row per wave (SoA) in the obstacle area
  R* wx = reinterpret_cast<R*>(lds + lds_head_bytes<R>()) + wave * 3 * 64;
  R* wy = wx + 64;
  R* wr = wy + 64;
  lds_prologue(S, lds, tid);
  __syncthreads();
  for (int k = wave; k < ne; k += kWaves) {
    const int e = e0 + k;
    if (io.mask && !io.mask[e]) continue;
    R rd0, rd1;
    R* last = S.sensor_last + (size_t)e * kSensors;
    if (S.I(I_SCAN)[e]) {
      R sp, cp;
      heading_sincos(S.F(F_PSI)[e], &sp, &cp);
      const int n = uniform(S.I(I_NOBS)[e]);
      if (l < S.cap) {
        const R* o = S.orow(e);
        wx[l] = o[l]; wy[l] = o[S.ostride + l]; wr[l] = o[2 * S.ostride + l];
      }
      Scan<R> sc;
      lidar_wave<R, kLidDefault>(RowSoA<R>{wx, wy, wr}, n, S.F(F_X)[e], S.F(F_Y)[e], sp, cp, rayoff,
                                 slots + wave * 128, marks + wave * 64, sc);
      rd0 = sc.rd0;
      rd1 = sc.rd1;
      last[l] = rd0;
      last[64 + l] = rd1;
    } else {
      rd0 = last[l];
      rd1 = last[64 + l];
    }
    float* row = io.obs + (size_t)e * kObsDim;
    row[kHdr + l] = (float)l_norm(rd0);
    row[kHdr + 64 + l] = (float)l_norm(rd1);
    R* info = io.info ? io.info + (size_t)e * USV_INFO_DIM : nullptr;
    if (S.np_reset) {
      if (l == 0) np_reset<R, MODE>(S, e, row, info, io.kpath);
    } else {
      const int ep = uniform(S.I(I_EPISODE)[e]);
      reset_wave<R, MODE>(S, e, row, info, io.kpath);
      if (S.exp) {
        __threadfence_block();                 // the wave's reset stores land before lane 0 rewrites
        if (l == 0) reset_experiment<R>(S, e, ep, row, info);
      }
    }
  }
}

// --------------------------------------------------------------------------- usv-asmc-v0
// Legacy UsvAsmcEnv (id usv-asmc-v0, usv_asmc_env.py:14-401): one 0.01 s ASMC + plant step per
// env step, lane-per-env, no lidar.  The reference stores its state as float32 after every
// step (:247-251) and builds T, CRB, CA, Dl, Dn, J as float32 arrays (:191-222); NumPy 2 keeps
// scalar arithmetic on float32 operands in float32.  Those rounding points are reproduced
// (q32 / float arithmetic) so the f64 build tracks the reference to float32 rounding; the
// first step after a reset runs on the float64 reset state (:258-300), flagged by elapsed == 0.
constexpr double kV0MinSpeed = 0.3, kV0KAk = 5.72, kV0KYe = 0.5, kV0SigmaYe = 1.0;
constexpr double kV0CAction = 1.0 / (((kPi / 2) / 2 - (-kPi / 2) / 2) / H * (((kPi / 2) / 2 - (-kPi / 2) / 2) / H));
constexpr double kV0WAction = 0.2, kV0TMin = -30.0, kV0TMax = 36.5;
constexpr int kFamV0 = 0, kFamYeInt = 1, kFamPid = 2;   // usv-asmc-v0, usv-asmc-ye-int-v0, usv-pid-v0

template <typename R> __device__ __forceinline__ R q32(R x) { return R((float)x); }

// sin / cos of the legacy path angle ak.  The legacy resets put the target on the start's line
// (yd = y0, usv_asmc_env.py:277-282), so ak = atan2(0, xd - x0) = +0 in every episode: a wave whose
// lanes all hold ak = 0 takes sin 0 = 0, cos 0 = 1 (the values libm returns) without the two libm calls.
template <typename R> __device__ __forceinline__ void v0_path_sincos(R ak, R& sa, R& ca) {
  if (__builtin_amdgcn_ballot_w64(ak != R(0)) == 0) { sa = R(0); ca = R(1); }
  else { sa = m_sin(ak); ca = m_cos(ak); }
}

template <typename R>
__device__ __forceinline__ void v0_obs(float* row, R u, R v_ak, R r, R ye, R psi_ak, R a_last) {
  row[0] = (float)u; row[1] = (float)v_ak; row[2] = (float)r;
  row[3] = (float)ye; row[4] = (float)psi_ak; row[5] = (float)a_last;
}

// UsvAsmcEnv.reset (usv_asmc_env.py:258-300); Philox draws replace np.random.uniform.
// FAM 1 / 2 are the float64 legacy envs on the same template: UsvAsmcYeIntEnv.reset
// (usv_asmc_ye_int_env.py:256-296: x, y ~ U(-5, 5), speed ~ U(0.4, 1.4)) and UsvPidEnv.reset
// (usv_pid_env.py:236-276: speed ~ U(0.4, 1.4)); the draw order is the same in all three.
// NumPy-exact mode: np.random.uniform on the legacy global RandomState (MT19937, seeded by
// np.random.seed), one lane per env, key[624] + pos kept in S.npmt.  uniform = lo + (hi - lo) *
// ((a >> 5) * 2^26 + (b >> 6)) / 2^53 over two 32-bit draws (numpy's mt19937 next_double).
struct NpMt {
  uint32_t* k;     // key word i of this env at k[i * stride]
  size_t stride;
  __device__ uint32_t& key(int i) const { return k[(size_t)i * stride]; }
  __device__ void twist() const {
    constexpr uint32_t kA = 0x9908b0dfu, kU = 0x80000000u, kL = 0x7fffffffu;
    int i = 0;
    for (; i < 624 - 397; ++i) {
      const uint32_t y = (key(i) & kU) | (key(i + 1) & kL);
      key(i) = key(i + 397) ^ (y >> 1) ^ ((0u - (y & 1u)) & kA);
    }
    for (; i < 623; ++i) {
      const uint32_t y = (key(i) & kU) | (key(i + 1) & kL);
      key(i) = key(i + 397 - 624) ^ (y >> 1) ^ ((0u - (y & 1u)) & kA);
    }
    const uint32_t y = (key(623) & kU) | (key(0) & kL);
    key(623) = key(396) ^ (y >> 1) ^ ((0u - (y & 1u)) & kA);
    key(624) = 0;
  }
  __device__ uint32_t next32() const {
    if (key(624) >= 624) twist();
    const uint32_t p = key(624);
    key(624) = p + 1;
    uint32_t y = key((int)p);
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }
  __device__ double uniform(double lo, double hi) const {
    const uint32_t a = next32() >> 5, b = next32() >> 6;
    return lo + (hi - lo) * ((a * 67108864.0 + b) / 9007199254740992.0);
  }
};

template <typename R, int FAM, typename G>
__device__ void v0_reset_draws(const State<R>& S, int e, float* row, int ep, G&& g);

template <typename R, int FAM = kFamV0>
__device__ void v0_reset(const State<R>& S, int e, float* row) {
  const int ep = S.I(I_EPISODE)[e];
  if (S.np_reset) {
    v0_reset_draws<R, FAM>(S, e, row, ep, NpMt{S.npmt + e, (size_t)S.fstride});
  } else {
    v0_reset_draws<R, FAM>(S, e, row, ep, Philox(S.seed, S.gid0 + (uint64_t)e, (uint32_t)ep));
  }
}

template <typename R, int FAM, typename G>
__device__ void v0_reset_draws(const State<R>& S, int e, float* row, int ep, G&& g) {
  const double lim = FAM == kFamYeInt ? 5.0 : 2.5;
  const double x = g.uniform(-lim, lim), y = g.uniform(-lim, lim);               // :260-261
  const double psi = g.uniform(-kPi, kPi);                                        // :262
  const double x0 = g.uniform(-2.5, 2.5), y0 = g.uniform(-2.5, 2.5);             // :275-276
  const double xd = g.uniform(15.0, 30.0), yd = y0;                              // :277-278
  const double ds = FAM == kFamV0 ? g.uniform(1.4, 2.4) : g.uniform(0.4, 1.4);   // :279
  const double ak = (double)(float)atan2(yd - y0, xd - x0);                       // :281-282
  const double psi_ak = (double)(float)wrap_once(psi - ak);                       // :284-286
  const double ye = -(x - x0) * sin(ak) + (y - y0) * cos(ak);                     // :287
  S.F(F_X)[e] = R(x); S.F(F_Y)[e] = R(y); S.F(F_PSI)[e] = R(psi);
  S.F(F_U)[e] = R(0); S.F(F_V)[e] = R(0); S.F(F_R)[e] = R(0);
  for (int i = 0; i < kV0Target; ++i) S.V(i)[e] = R(0);                          // last, aux
  const double tg[6] = {x0, y0, ds, ak, xd, yd};
  for (int i = 0; i < 6; ++i) S.V(kV0Target + i)[e] = R(tg[i]);
  S.V(kV0ALast)[e] = R(0);
  S.V(kV0Ye)[e] = R(0); S.V(kV0Ye + 1)[e] = R(0);                                 // ye_int, ye_last
  S.I(I_ELAPSED)[e] = 0;
  S.I(I_EPISODE)[e] = ep + 1;
  v0_obs<R>(row, R(0), R(0), R(0), R(ye), R(psi_ak), R(0));                      // :289-298
}

template <typename R>
__global__ __launch_bounds__(kBlock) void v0_step_kernel(State<R> S, IO<R> io) {
  const int e = blockIdx.x * kBlock + threadIdx.x;
  if (e >= S.N) return;
  const bool first = S.I(I_ELAPSED)[e] == 0;        // reference state still float64 (reset arrays)
  const float af = io.act[e];
  const R a = R(af);
  R u = S.F(F_U)[e], v = S.F(F_V)[e], r = S.F(F_R)[e];
  R x = S.F(F_X)[e], y = S.F(F_Y)[e], psi = S.F(F_PSI)[e];
  R e_u_int = S.V(kV0Aux)[e], ka_u = S.V(kV0Aux + 1)[e], ka_psi = S.V(kV0Aux + 2)[e];
  const R xd_l = S.V(0)[e], yd_l = S.V(1)[e], pd_l = S.V(2)[e];
  const R ud_l = S.V(3)[e], vd_l = S.V(4)[e], rd_l = S.V(5)[e];
  const R e_u_last = S.V(6)[e], kdu_l = S.V(7)[e], kdp_l = S.V(8)[e];
  const R x0 = S.V(kV0Target)[e], y0 = S.V(kV0Target + 1)[e], ds = S.V(kV0Target + 2)[e];
  const R ak = S.V(kV0Target + 3)[e];
  const R a_last = S.V(kV0ALast)[e];
  // action_dot (:120): float32 arithmetic once the stored state is float32
  const R action_dot = first ? (a - a_last) / R(H) : R((af - (float)a_last) / (float)H);
  const R psi_d = wrap_once(a + ak);                                             // :123-124
  const bool fast = m_abs(u) > R(1.2);                                           // :126-130
  const R xu = fast ? R(64.55) : R(-25.0), xuu = fast ? R(-70.92) : R(0.0);
  // hydrodynamic terms, f, C, D: float32 (state is float32; exactly 0 on the first step)
  const float uf = (float)u, vf = (float)v, rf = (float)r;
  const float mag = sqrtf(uf * uf + vf * vf);
  const float yv = (0.5f * (-40000.0f * fabsf(vf))) *
                   (float)(1.1 + 0.0045 * (1.01 / 0.09) - 0.1 * (0.27 / 0.09) + 0.016 * ((0.27 / 0.09) * (0.27 / 0.09)));  // :132
  const float yr = (((float)(6 * (-3.141592 * 1000)) * mag) * 0.09f) * 0.09f * 1.01f;            // :134
  const float nv = (((float)(0.06 * (-3.141592 * 1000)) * mag) * 0.09f) * 0.09f * 1.01f;         // :136
  const float nr = (((float)(0.02 * (-3.141592 * 1000)) * mag) * 0.09f) * 0.09f * 1.01f * 1.01f; // :138
  const float fu = ((float)(MASS - Y_V_DOT) * vf * rf + ((float)xuu * fabsf(uf) + (float)xu * uf)) / (float)(MASS - X_U_DOT);  // :144
  const float fpsi = ((float)(-X_U_DOT + Y_V_DOT) * uf * vf + (nr * rf)) / (float)(IZ - N_R_DOT);                             // :145
  const R e_psi = wrap_once(psi_d - psi);                                        // :147-148
  const R e_psi_dot = R(0) - r;                                                  // :149
  const R u_psi = R(1) / (R(1) + m_exp(R(10) * (m_abs(e_psi) * R(2 / kPi) - R(0.5))));  // :153
  const R u_d = (ds - R(kV0MinSpeed)) * u_psi + R(kV0MinSpeed);                  // :155-156
  const R e_u = u_d - u;                                                         // :158
  e_u_int = R(H) * (e_u + e_u_last) / R(2) + e_u_int;                            // :159 (e_u_last stale)
  const R sig_u = e_u + R(LAMBDA_U) * e_u_int;                                   // :161
  const R sig_p = e_psi_dot + R(LAMBDA_PSI) * e_psi;                             // :162
  const R kdu = ka_u > R(KMIN_U) ? R(K_U) * m_sign(m_abs(sig_u) - R(MU_U)) : R(KMIN_U);       // :164
  const R kdp = ka_psi > R(KMIN_PSI) ? R(K_PSI) * m_sign(m_abs(sig_p) - R(MU_PSI)) : R(KMIN_PSI);
  ka_u = R(H) * (kdu + kdu_l) / R(2) + ka_u;                                     // :167
  ka_psi = R(H) * (kdp + kdp_l) / R(2) + ka_psi;                                 // :170
  const R ua_u = -ka_u * m_sqrt(m_abs(sig_u)) * m_sign(sig_u) - R(K2_U) * sig_u;           // :173
  const R ua_p = -ka_psi * m_sqrt(m_abs(sig_p)) * m_sign(sig_p) - R(K2_PSI) * sig_p;       // :174
  const R tx = (R(LAMBDA_U) * e_u - R(fu) - ua_u) / R(1.0 / (MASS - X_U_DOT));  // :176
  const R tz = (R(LAMBDA_PSI) * e_psi - R(fpsi) - ua_p) / R(1.0 / (IZ - N_R_DOT));
  const R tport = m_clip(tx / R(2) + tz / R(B_TH), R(kV0TMin), R(kV0TMax));      // :179-185
  const R tstbd = m_clip(tx / R(2 * C_TH) - tz / R(B_TH * C_TH), R(kV0TMin), R(kV0TMax));
  const float t0 = (float)(tport + R(C_TH) * tstbd);                             // :191 float32 T
  const float t2 = (float)(R(0.5 * B_TH) * (tport - R(C_TH) * tstbd));
  // C = CRB + CA, D = Dl - Dn as float32 (:193-212)
  const float c02 = (0.0f - 30.0f * vf) + 2.0f * ((float)Y_V_DOT * vf + (float)((Y_R_DOT + N_V_DOT) / 2) * rf);
  const float c12 = (30.0f * uf) + (0.0f - (float)(X_U_DOT * MASS) * uf);
  const float c20 = (30.0f * vf) + 2.0f * (((float)(0 - Y_V_DOT) * vf) - (float)((Y_R_DOT + N_V_DOT) / 2) * rf);
  const float c21 = (0.0f - 30.0f * uf) + ((float)(X_U_DOT * MASS) * uf);
  const float av = fabsf(vf), ar = fabsf(rf);
  const float d00 = (float)(0 - xu) - (float)(xuu * m_abs(u));
  const float d11 = (0.0f - yv) - ((float)YVV * av + (float)YVR * ar);
  const float d12 = (0.0f - yr) - ((float)YRV * av + (float)YRR * ar);
  const float d21 = (0.0f - nv) - ((float)NVV * av + (float)NVR * ar);
  const float d22 = (0.0f - nr) - ((float)NRV * av + (float)NRR * ar);
  // T - C nu - D nu (:214-215), float32 (nu is float32 after the first step, 0 on it)
  const float rhs0 = (t0 - c02 * rf) - d00 * uf;
  const float rhs1 = (0.0f - c12 * rf) - (d11 * vf + d12 * rf);
  const float rhs2 = (t2 - (c20 * uf + c21 * vf)) - (d21 * vf + d22 * rf);
  const R ud = R(MI00) * R(rhs0);                                                // :214 M^-1 (f64)
  const R vd = R(MI11) * R(rhs1) + R(MI12) * R(rhs2);
  const R rd = R(MI21) * R(rhs1) + R(MI22) * R(rhs2);
  u = R(H) * (ud + ud_l) / R(2) + u;                                             // :216-217
  v = R(H) * (vd + vd_l) / R(2) + v;
  r = R(H) * (rd + rd_l) / R(2) + r;
  // J as float32 (:220-222): of the float32 heading, or the float64 reset heading rounded
  const R cj = first ? R((float)m_cos(psi)) : R(cosf((float)psi));
  const R sj = first ? R((float)m_sin(psi)) : R(sinf((float)psi));
  const R xd = cj * u - sj * v, yd = sj * u + cj * v, pd = r;                    // :224
  x = R(H) * (xd + xd_l) / R(2) + x;                                             // :225
  y = R(H) * (yd + yd_l) / R(2) + y;
  psi = wrap_once(R(H) * (pd + pd_l) / R(2) + psi);                              // :228-229
  const R psi_ak = wrap_once(psi - ak);                                          // :231-232
  R sak, cak;
  v0_path_sincos(ak, sak, cak);
  const R ye = -(x - x0) * sak + (y - y0) * cak;                                 // :234
  const R ye_abs = m_abs(ye);
  // compute_reward (:364-374)
  const R pa = m_abs(psi_ak);
  const R cad = first ? R(-kV0CAction) * (action_dot * action_dot)
                      : R((float)(-kV0CAction) * ((float)action_dot * (float)action_dot));
  const R r_act = R(kV0WAction) * tanh(cad);
  const R r_ye = ye_abs > R(kV0SigmaYe) ? m_exp(R(-kV0KYe) * ye_abs) : m_exp(R(-kV0KYe) * (ye_abs * ye_abs) / R(kV0SigmaYe));
  const R r_ak = -m_exp(R(kV0KAk) * (pa - R(kPi)));
  const R v_ak = m_sin(psi_ak) * u + m_cos(psi_ak) * v;                          // body_to_path :376-390
  const bool done = ye_abs > R(10) || m_abs(x) > R(30);                          // :241-245
  const int el = S.I(I_ELAPSED)[e] + 1;
  const bool trunc = !done && S.limit > 0 && el >= S.limit;
  io.rew[e] = done ? R(-1) : (pa < R(kPi / 2) ? r_act + r_ye : r_ak);
  io.term[e] = done;
  io.trunc[e] = trunc;
  if (io.done) io.done[e] = done | trunc;
  float* row = io.obs + (size_t)e * 6;
  // stored state (float32, :247-251)
  S.F(F_U)[e] = q32(u); S.F(F_V)[e] = q32(v); S.F(F_R)[e] = q32(r);
  S.F(F_X)[e] = q32(x); S.F(F_Y)[e] = q32(y); S.F(F_PSI)[e] = q32(psi);
  S.V(kV0Aux)[e] = q32(e_u_int); S.V(kV0Aux + 1)[e] = q32(ka_u); S.V(kV0Aux + 2)[e] = q32(ka_psi);
  S.V(0)[e] = q32(xd); S.V(1)[e] = q32(yd); S.V(2)[e] = q32(pd);
  S.V(3)[e] = q32(ud); S.V(4)[e] = q32(vd); S.V(5)[e] = q32(rd);
  S.V(6)[e] = q32(e_u_last); S.V(7)[e] = q32(kdu); S.V(8)[e] = q32(kdp);
  S.V(kV0ALast)[e] = a;
  S.I(I_ELAPSED)[e] = el;
  v0_obs<R>(row, u, v_ak, r, ye, psi_ak, a);
  if (done || trunc) {
    if (io.fobs) v0_obs<R>(io.fobs + (size_t)e * 6, u, v_ak, r, ye, psi_ak, a);
    if (S.autoreset == USV_AUTORESET_SAME_STEP) v0_reset<R, kFamV0>(S, e, row);
  }
}

template <typename R, int FAM>
__global__ __launch_bounds__(kBlock) void v0_reset_kernel(State<R> S, IO<R> io) {
  const int e = blockIdx.x * kBlock + threadIdx.x;
  if (e >= S.N || (io.mask && !io.mask[e])) return;
  v0_reset<R, FAM>(S, e, io.obs + (size_t)e * 6);
}

// --------------------------------------------------------------------------- float64 legacy family
// UsvAsmcYeIntEnv (usv-asmc-ye-int-v0, usv_asmc_ye_int_env.py:92-253) and UsvPidEnv (usv-pid-v0,
// usv_pid_env.py:89-233): the usv-asmc-v0 plant with the state kept in float64 (no float32
// arrays), so the whole step runs in R.  Lane per env.  Statement order follows the reference
// (contraction is off in this translation unit), so the f64 build tracks it to libm ulps.
// Citations are usv_asmc_ye_int_env.py lines; usv_pid_env.py has the same statements 4 lines
// earlier (its control law: :148-155).
constexpr double kYeIntKI = 0.001;                                               // ye_int :51
constexpr double kPidKpU = 1.1, kPidKiU = 0.2, kPidKdU = 0.1, kPidKpPsi = 0.8, kPidKdPsi = 3.0;  // pid :40-44
constexpr double kYvK = 1.1 + 0.0045 * (1.01 / 0.09) - 0.1 * (0.27 / 0.09) + 0.016 * ((0.27 / 0.09) * (0.27 / 0.09));

template <typename R, int FAM>
__global__ __launch_bounds__(kBlock) void legacy_step_kernel(State<R> S, IO<R> io) {
  const int e = blockIdx.x * kBlock + threadIdx.x;
  if (e >= S.N) return;
  const R a = R(io.act[e]);
  R u = S.F(F_U)[e], v = S.F(F_V)[e], r = S.F(F_R)[e];
  R x = S.F(F_X)[e], y = S.F(F_Y)[e], psi = S.F(F_PSI)[e];
  R e_u_int = S.V(kV0Aux)[e], ka_u = S.V(kV0Aux + 1)[e], ka_psi = S.V(kV0Aux + 2)[e];
  const R xd_l = S.V(0)[e], yd_l = S.V(1)[e], pd_l = S.V(2)[e];
  const R ud_l = S.V(3)[e], vd_l = S.V(4)[e], rd_l = S.V(5)[e];
  const R e_u_last = S.V(6)[e];
  R kdu = S.V(7)[e], kdp = S.V(8)[e];
  const R x0 = S.V(kV0Target)[e], y0 = S.V(kV0Target + 1)[e], ds = S.V(kV0Target + 2)[e];
  const R ak = S.V(kV0Target + 3)[e];
  const R action_dot = (a - S.V(kV0ALast)[e]) / R(H);                           // :113
  const R psi_d = wrap_once(a + ak);                                             // :116-117
  const bool fast = m_abs(u) > R(1.2);                                           // :119-123
  const R xu = fast ? R(64.55) : R(-25.0), xuu = fast ? R(-70.92) : R(0.0);
  const R mag = m_sqrt(u * u + v * v);                                           // :125-132
  const R yv = (R(0.5) * (R(-40 * 1000) * m_abs(v))) * R(kYvK);
  const R yr = (((R(6 * (-3.141592 * 1000)) * mag) * R(0.09)) * R(0.09)) * R(1.01);
  const R nv = (((R(0.06 * (-3.141592 * 1000)) * mag) * R(0.09)) * R(0.09)) * R(1.01);
  const R nr = ((((R(0.02 * (-3.141592 * 1000)) * mag) * R(0.09)) * R(0.09)) * R(1.01)) * R(1.01);
  const R f_u = ((R(MASS - Y_V_DOT) * v * r) + (xuu * m_abs(u) + xu * u)) / R(MASS - X_U_DOT);    // :137
  const R f_psi = ((R(-X_U_DOT + Y_V_DOT) * u * v) + (nr * r)) / R(IZ - N_R_DOT);                 // :138
  const R e_psi = wrap_once(psi_d - psi);                                        // :140-141
  const R e_psi_dot = R(0) - r;                                                  // :142
  const R u_psi = R(1) / (R(1) + m_exp(R(10) * (m_abs(e_psi) * R(2 / kPi) - R(0.5))));  // :146
  const R u_d = (ds - R(kV0MinSpeed)) * u_psi + R(kV0MinSpeed);                  // :148-149
  const R e_u = u_d - u;                                                         // :151
  e_u_int = R(H) * (e_u + e_u_last) / R(2) + e_u_int;                            // :152 (e_u_last stale)
  R tx, tz;
  if constexpr (FAM == kFamYeInt) {                                              // ASMC :154-170
    const R sig_u = e_u + R(LAMBDA_U) * e_u_int;
    const R sig_p = e_psi_dot + R(LAMBDA_PSI) * e_psi;
    const R kdu_n = ka_u > R(KMIN_U) ? R(K_U) * m_sign(m_abs(sig_u) - R(MU_U)) : R(KMIN_U);
    const R kdp_n = ka_psi > R(KMIN_PSI) ? R(K_PSI) * m_sign(m_abs(sig_p) - R(MU_PSI)) : R(KMIN_PSI);
    ka_u = R(H) * (kdu_n + kdu) / R(2) + ka_u;
    ka_psi = R(H) * (kdp_n + kdp) / R(2) + ka_psi;
    kdu = kdu_n; kdp = kdp_n;
    const R ua_u = (-ka_u * m_sqrt(m_abs(sig_u)) * m_sign(sig_u)) - R(K2_U) * sig_u;
    const R ua_p = (-ka_psi * m_sqrt(m_abs(sig_p)) * m_sign(sig_p)) - R(K2_PSI) * sig_p;
    tx = ((R(LAMBDA_U) * e_u) - f_u - ua_u) / R(1.0 / (MASS - X_U_DOT));
    tz = ((R(LAMBDA_PSI) * e_psi) - f_psi - ua_p) / R(1.0 / (IZ - N_R_DOT));
  } else {                                                                       // PID, pid :148-155
    const R e_u_dot = (e_u - e_u_last) / R(H);
    const R ua_u = (R(kPidKpU) * e_u) + (R(kPidKiU) * e_u_int) + (R(kPidKdU) * e_u_dot);
    const R ua_p = (R(kPidKpPsi) * e_psi) + (R(kPidKdPsi) * e_psi_dot);
    tx = (-f_u + ua_u) / R(1.0 / (MASS - X_U_DOT));
    tz = (-f_psi + ua_p) / R(1.0 / (IZ - N_R_DOT));
  }
  R tport = tx / R(2) + tz / R(B_TH);                                            // :172-178
  R tstbd = tx / R(2 * C_TH) - tz / R(B_TH * C_TH);
  tport = tport > R(kV0TMax) ? R(kV0TMax) : tport;
  tport = tport < R(kV0TMin) ? R(kV0TMin) : tport;
  tstbd = tstbd > R(kV0TMax) ? R(kV0TMax) : tstbd;
  tstbd = tstbd < R(kV0TMin) ? R(kV0TMin) : tstbd;
  const R t0 = tport + R(C_TH) * tstbd;                                          // :184
  const R t2 = R(0.5 * B_TH) * (tport - R(C_TH) * tstbd);
  // C = CRB + CA, D = Dl - Dn (:186-205): their non-zero entries
  const R c02 = (R(0) - R(MASS) * v) + R(2) * ((R(Y_V_DOT) * v) + R((Y_R_DOT + N_V_DOT) / 2) * r);
  const R c12 = (R(MASS) * u) + (R(0) - R(X_U_DOT * MASS) * u);
  const R c20 = (R(MASS) * v) + R(2) * ((R(0 - Y_V_DOT) * v) - R((Y_R_DOT + N_V_DOT) / 2) * r);
  const R c21 = (R(0) - R(MASS) * u) + (R(X_U_DOT * MASS) * u);
  const R av = m_abs(v), ar = m_abs(r);
  const R d00 = (R(0) - xu) - xuu * m_abs(u);
  const R d11 = (R(0) - yv) - (R(YVV) * av + R(YVR) * ar);
  const R d12 = (R(0) - yr) - (R(YRV) * av + R(YRR) * ar);
  const R d21 = (R(0) - nv) - (R(NVV) * av + R(NVR) * ar);
  const R d22 = (R(0) - nr) - (R(NRV) * av + R(NRR) * ar);
  const R rhs0 = (t0 - c02 * r) - d00 * u;                                       // :207-208
  const R rhs1 = (R(0) - c12 * r) - (d11 * v + d12 * r);
  const R rhs2 = (t2 - (c20 * u + c21 * v)) - (d21 * v + d22 * r);
  const R ud = R(MI00) * rhs0;                                                   // M^-1 (block form)
  const R vd = R(MI11) * rhs1 + R(MI12) * rhs2;
  const R rd = R(MI21) * rhs1 + R(MI22) * rhs2;
  u = R(H) * (ud + ud_l) / R(2) + u;                                             // :209-211
  v = R(H) * (vd + vd_l) / R(2) + v;
  r = R(H) * (rd + rd_l) / R(2) + r;
  const R cj = m_cos(psi), sj = m_sin(psi);                                      // J(psi) :213-215
  const R xd = cj * u - sj * v, yd = sj * u + cj * v, pd = r;
  x = R(H) * (xd + xd_l) / R(2) + x;                                             // :217-219
  y = R(H) * (yd + yd_l) / R(2) + y;
  psi = wrap_once(R(H) * (pd + pd_l) / R(2) + psi);                              // :221-222
  const R psi_ak = wrap_once(psi - ak);                                          // :224-225
  R sak, cak;
  v0_path_sincos(ak, sak, cak);
  const R ye = -(x - x0) * sak + (y - y0) * cak;                                 // :227
  const R ye_abs = m_abs(ye);
  const R pa = m_abs(psi_ak);
  const R r_act = R(kV0WAction) * tanh(R(-kV0CAction) * (action_dot * action_dot));
  const R r_ak = -m_exp(R(kV0KAk) * (pa - R(kPi)));
  R ye_obs = ye, reward;
  if constexpr (FAM == kFamYeInt) {
    R ye_int = S.V(kV0Ye)[e];
    const R ye_last = S.V(kV0Ye + 1)[e];
    if (m_sign(ye) != m_sign(ye_last)) ye_int = R(0);                            // :230-231
    ye_int = R(H) * (ye + ye_last) + ye_int;                                     // :232
    ye_obs = ye + R(kYeIntKI) * ye_int;                                          // ye_ss :235
    S.V(kV0Ye)[e] = ye_int;
    S.V(kV0Ye + 1)[e] = ye;
    reward = r_act + (pa < R(kPi / 2) ? m_exp(R(-kV0KYe) * ye_abs) : r_ak);      // :350-360
  } else {
    const R r_ye = ye_abs > R(kV0SigmaYe) ? m_exp(R(-kV0KYe) * ye_abs)
                                          : m_exp(R(-kV0KYe) * (ye_abs * ye_abs) / R(kV0SigmaYe));
    reward = pa < R(kPi / 2) ? r_act + r_ye : r_ak;                              // pid :329-338
  }
  const R v_ak = m_sin(psi_ak) * u + m_cos(psi_ak) * v;                          // body_to_path :239
  const bool done = ye_abs > R(10) || x < R(-10);                                // :241-245
  const int el = S.I(I_ELAPSED)[e] + 1;
  const bool trunc = !done && S.limit > 0 && el >= S.limit;
  io.rew[e] = done ? R(-1) : reward;
  io.term[e] = done;
  io.trunc[e] = trunc;
  if (io.done) io.done[e] = done | trunc;
  S.F(F_U)[e] = u; S.F(F_V)[e] = v; S.F(F_R)[e] = r;                             // :247-251
  S.F(F_X)[e] = x; S.F(F_Y)[e] = y; S.F(F_PSI)[e] = psi;
  S.V(kV0Aux)[e] = e_u_int; S.V(kV0Aux + 1)[e] = ka_u; S.V(kV0Aux + 2)[e] = ka_psi;
  S.V(0)[e] = xd; S.V(1)[e] = yd; S.V(2)[e] = pd;
  S.V(3)[e] = ud; S.V(4)[e] = vd; S.V(5)[e] = rd;
  S.V(7)[e] = kdu; S.V(8)[e] = kdp;
  S.V(kV0ALast)[e] = a;
  S.I(I_ELAPSED)[e] = el;
  float* row = io.obs + (size_t)e * 6;
  v0_obs<R>(row, u, v_ak, r, ye_obs, psi_ak, a);
  if (done || trunc) {
    if (io.fobs) v0_obs<R>(io.fobs + (size_t)e * 6, u, v_ak, r, ye_obs, psi_ak, a);
    if (S.autoreset == USV_AUTORESET_SAME_STEP) v0_reset<R, FAM>(S, e, row);
  }
}

}  // namespace usv

// ============================================================================= host side
using namespace usv;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                 \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess)                                                             \
      return fail(USV_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(_e));      \
  } while (0)

struct FieldDesc { const char* name; int is_int; };
const FieldDesc kFields[USV_FIELD_COUNT] = {
    {"x", 0}, {"y", 0}, {"psi", 0}, {"u", 0}, {"v", 0}, {"r", 0}, {"last_u", 0}, {"last_r", 0},
    {"progress", 0}, {"path_x0", 0}, {"path_y0", 0}, {"path_x1", 0}, {"path_y1", 0},
    {"max_u", 0}, {"max_r", 0}, {"ref_v", 0}, {"n_obs", 1}, {"elapsed", 1}, {"episode", 1},
    {"scan_valid", 1}, {"obs_x", 0}, {"obs_y", 0}, {"obs_r", 0}, {"sensor_last", 0}, {"asmc", 0},
    {"v0_last", 0}, {"v0_aux", 0}, {"v0_target", 0}, {"v0_action_last", 0}, {"v0_ye", 0}, {"np_rng", 1}, {"np_mt", 1}};

bool is_legacy(int mode) {   // lane-per-env legacy envs: obs 6, scalar action, no lidar
  return mode == USV_MODE_ASMC_V0 || mode == USV_MODE_ASMC_YE_INT_V0 || mode == USV_MODE_PID_V0;
}

struct Handle {
  usv_config cfg;
  int device;
  // step-kernel variant (see launch_step; all variants give identical results):
  //   kind 0 = block kernel (one dynamics wave per block, barriers), 1 = fused wave kernel
  //   (step_kernel_wave), 2 = split (dyn_kernel + scan_kernel); epb = envs per 256-thread block
  //   4 / 5 = block-queue step, split / fused (step_q_kernel; f32 window lidar, cap <= 32)
  int epb = 64, lid = 7, kind = 1;
  int prio = 1;                        // scan loops raise the priority of lagging waves
  int cus = 256;                       // compute units of the device (State::qyoung)
  void* slab = nullptr;
  void* exp_buf = nullptr;             // device usv_experiment record (kExp* layout, in R)
  State<float> sf{};
  State<double> sd{};
};

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

template <typename R>
int carve(Handle* h, State<R>& S) {
  const size_t N = (size_t)h->cfg.num_envs, cap = (size_t)h->cfg.obstacle_cap;
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t stride = al(N * sizeof(R)) / sizeof(R);   // also >= N int32 (sizeof(R) >= 4)
  const size_t bytes = F_NREAL * stride * sizeof(R) + al(I_NINT * stride * 4) +
                       al(N * 3 * obst_stride((int)cap) * sizeof(R)) + al(N * kSensors * sizeof(R)) +
                       al((size_t)kAsmcN * N * sizeof(R)) + al((size_t)kV0N * stride * sizeof(R)) +
                       al(2 * kSensors * sizeof(R)) + al(2 * N * sizeof(R4<R>)) + al(10 * stride * 4) +
                       al((kExpObs + 3 * cap) * sizeof(R)) + al(N * kQRec * sizeof(float)) +
                       (is_legacy(h->cfg.mode) ? al(625 * stride * 4) : 0);
  HIP_TRY(hipMalloc(&h->slab, bytes));
  HIP_TRY(hipMemset(h->slab, 0, bytes));
  char* p = (char*)h->slab;
  auto take = [&](size_t b) { char* q = p; p += al(b); return (void*)q; };
  S.freal = (R*)take(F_NREAL * stride * sizeof(R));
  S.fint = (int32_t*)take(I_NINT * stride * 4);
  S.fstride = (int)stride;
  S.ostride = obst_stride((int)cap);
  S.obst = (R*)take(N * 3 * S.ostride * sizeof(R));
  S.sensor_last = (R*)take(N * kSensors * sizeof(R));
  S.asmc = (R*)take((size_t)kAsmcN * N * sizeof(R));
  S.v0 = (R*)take((size_t)kV0N * stride * sizeof(R));
  R* tab = (R*)take(2 * kSensors * sizeof(R));
  S.ray_tab = tab;
  S.pose = (R4<R>*)take(2 * N * sizeof(R4<R>));
  S.qrec = (float*)take(N * kQRec * sizeof(float));
  S.nprng = (uint32_t*)take(10 * stride * 4);
  h->exp_buf = take((kExpObs + 3 * cap) * sizeof(R));
  S.exp = nullptr;                                       // usv_set_experiment installs it
  S.perturb = (h->cfg.flags & USV_FLAG_PERTURB) != 0;
  S.npmt = is_legacy(h->cfg.mode) ? (uint32_t*)take(625 * stride * 4) : nullptr;   // legacy ids only
  S.np_reset = 0;
  S.N = h->cfg.num_envs;
  S.cap = h->cfg.obstacle_cap;
  S.limit = h->cfg.max_episode_steps;
  S.autoreset = h->cfg.autoreset;
  S.prio = h->prio;
  S.rowspan = h->cfg.num_envs >= kRowSpanFrom;
  S.qyoung = INT_MAX;                                    // (set per launch: launch_step)
  S.seed = h->cfg.seed;
  S.gid0 = h->cfg.env_id_offset;
  // ray offsets start + i*res (usv_asmc_ca_env.py:420), cos/sin in float64 on the host
  std::vector<R> ht(2 * kSensors);
  const double span = (2.0 / 3.0) * (2.0 * kPi), res = span / kSensors;
  for (int i = 0; i < kSensors; ++i) {
    const double a = i * res;            // from ray 0 (heading - 120 deg): see to_ray0
    ht[2 * i] = (R)std::cos(a);          // interleaved (c, s): the LDS image, copied verbatim
    ht[2 * i + 1] = (R)std::sin(a);
  }
  HIP_TRY(hipMemcpy(tab, ht.data(), 2 * kSensors * sizeof(R), hipMemcpyHostToDevice));
  // reference __init__ defaults: max_action = [3, 0, 3] (simple_env.py:32)
  std::vector<R> three(N, (R)3);
  HIP_TRY(hipMemcpy(S.F(F_MAX_U), three.data(), N * sizeof(R), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(S.F(F_MAX_R), three.data(), N * sizeof(R), hipMemcpyHostToDevice));
  return USV_OK;
}

// Step-kernel variants: envs per block x lidar variant.  Selected per handle at create time
// (USV_STEP_VARIANT="epb,lid" overrides, for tuning sweeps); all variants are bit-identical.

template <typename R, int MODE, int EPW>
void* pick_wave_lid(int lid) {
  if constexpr (std::is_same<R, float>::value && MODE == USV_MODE_SIMPLE) {
    if (lid == 0) return (void*)&step_kernel_wave_tight<R, MODE, EPW, 0>;
    if (lid == 3) return (void*)&step_kernel_wave_tight<R, MODE, EPW, 3>;
    return (void*)&step_kernel_wave_tight<R, MODE, EPW, 7>;
  }
  if (lid == 0) return (void*)&step_kernel_wave<R, MODE, EPW, 0>;
  if (lid == 3) return (void*)&step_kernel_wave<R, MODE, EPW, 3>;
  return (void*)&step_kernel_wave<R, MODE, EPW, 7>;
}
template <typename R, int MODE>
void* pick_wave(int epw, int lid, size_t* lds, int cap) {
  *lds = lds_scan_bytes<R>(cap);
  if (epw == 4) return pick_wave_lid<R, MODE, 4>(lid);
  if (epw == 16) return pick_wave_lid<R, MODE, 16>(lid);
  return pick_wave_lid<R, MODE, 8>(lid);
}

template <typename R, int MODE, int EPW, int WPB>
void* pick_scan_lid(int lid) {
  if constexpr (std::is_same<R, float>::value && MODE == USV_MODE_SIMPLE) {
    if (lid == 0) return (void*)&scan_kernel_tight<R, MODE, EPW, 0, WPB>;
    if (lid == 3) return (void*)&scan_kernel_tight<R, MODE, EPW, 3, WPB>;
    return (void*)&scan_kernel_tight<R, MODE, EPW, 7, WPB>;
  }
  if constexpr (std::is_same<R, double>::value) {
    if (lid == 7) return (void*)&scan_kernel_d<R, MODE, EPW, 7, WPB>;
  }
  if (lid == 0) return (void*)&scan_kernel<R, MODE, EPW, 0, WPB>;
  if (lid == 3) return (void*)&scan_kernel<R, MODE, EPW, 3, WPB>;
  return (void*)&scan_kernel<R, MODE, EPW, 7, WPB>;
}
template <typename R, int MODE, int WPB>
void* pick_scan(int epw, int lid) {
  if (epw == 2) return pick_scan_lid<R, MODE, 2, WPB>(lid);
  if (epw == 8) return pick_scan_lid<R, MODE, 8, WPB>(lid);
  if constexpr (std::is_same<R, double>::value && WPB == 4)
    if (epw == 16) return pick_scan_lid<R, MODE, 16, WPB>(lid);   // f64: one round of waves at 65 536 envs
  return pick_scan_lid<R, MODE, 4, WPB>(lid);
}

// split_chain (kind 6, usv-asmc-simple): the fused q kernel without the ASMC chain in its phase 1;
// info: the fused kernels' info-row instantiation (the split kind 4 writes info in dyn_rec_kernel)
template <bool DONE, bool INFO>
void* pick_q_done(int mode, bool fused, bool small, bool split_chain, bool span) {
  const bool simple = mode == USV_MODE_SIMPLE;
  if constexpr (!INFO)
    if (span && fused && !small) {                     // row-span stores (State::rowspan)
      if (simple) return (void*)&step_q_kernel<USV_MODE_SIMPLE, true, DONE, true, false, true>;
      return split_chain ? (void*)&step_q_kernel<USV_MODE_ASMC_SIMPLE, true, DONE, false, false, true>
                         : (void*)&step_q_kernel<USV_MODE_ASMC_SIMPLE, true, DONE, true, false, true>;
    }
  if (!simple && split_chain)
    return small ? (void*)&step_qs_kernel<USV_MODE_ASMC_SIMPLE, DONE, false, INFO>
                 : (void*)&step_q_kernel<USV_MODE_ASMC_SIMPLE, true, DONE, false, INFO>;
  if (small) return simple ? (void*)&step_qs_kernel<USV_MODE_SIMPLE, DONE, true, INFO>
                           : (void*)&step_qs_kernel<USV_MODE_ASMC_SIMPLE, DONE, true, INFO>;
  if (fused) return simple ? (void*)&step_q_kernel<USV_MODE_SIMPLE, true, DONE, true, INFO>
                           : (void*)&step_q_kernel<USV_MODE_ASMC_SIMPLE, true, DONE, true, INFO>;
  return simple ? (void*)&step_q_kernel<USV_MODE_SIMPLE, false, DONE> : (void*)&step_q_kernel<USV_MODE_ASMC_SIMPLE, false, DONE>;
}
void* pick_q(int mode, bool fused, bool small = false, bool done = false, bool split_chain = false, bool info = false,
             bool span = false) {
  if (info && fused)
    return done ? pick_q_done<true, true>(mode, fused, small, split_chain, span)
                : pick_q_done<false, true>(mode, fused, small, split_chain, span);
  return done ? pick_q_done<true, false>(mode, fused, small, split_chain, span)
              : pick_q_done<false, false>(mode, fused, small, split_chain, span);
}

template <typename R>
int launch_step_kernels(Handle* h, State<R>& S, const float* act, float* obs, void* rew, uint8_t* term,
                        uint8_t* trunc, uint8_t* done, float* fobs, void* info, hipStream_t st);

// The step, then (NumPy-exact reset mode) the resets of the envs that ended in it.
template <typename R>
int launch_step(Handle* h, State<R>& S, const float* act, float* obs, void* rew, uint8_t* term,
                uint8_t* trunc, uint8_t* done, float* fobs, void* info, hipStream_t st) {
  const int rc = launch_step_kernels(h, S, act, obs, rew, term, trunc, done, fobs, info, st);
  // (the legacy kernels reset inline, from the MT19937 state, in the NumPy-exact mode too)
  if (rc != USV_OK || S.autoreset != USV_AUTORESET_SAME_STEP || is_legacy(h->cfg.mode)) return rc;
  IO<R> io{act, obs, (R*)rew, term, trunc, fobs, nullptr, nullptr, 0};
  const dim3 grid((S.N + kBlock - 1) / kBlock), block(kBlock);
  if (!S.np_reset) {
    if (S.exp) hipLaunchKernelGGL((exp_autoreset_kernel<R>), grid, block, 0, st, S, io);
    HIP_TRY(hipGetLastError());
    return USV_OK;
  }
  if (h->cfg.mode == USV_MODE_SIMPLE)
    hipLaunchKernelGGL((np_autoreset_kernel<R, USV_MODE_SIMPLE>), grid, block, 0, st, S, io);
  else
    hipLaunchKernelGGL((np_autoreset_kernel<R, USV_MODE_ASMC_SIMPLE>), grid, block, 0, st, S, io);
  HIP_TRY(hipGetLastError());
  return USV_OK;
}

template <typename R>
int launch_step_kernels(Handle* h, State<R>& S, const float* act, float* obs, void* rew, uint8_t* term,
                        uint8_t* trunc, uint8_t* done, float* fobs, void* info, hipStream_t st) {
  IO<R> io{act, obs, (R*)rew, term, trunc, fobs, nullptr, is_legacy(h->cfg.mode) ? nullptr : (R*)info, 0, done};
  if (is_legacy(h->cfg.mode)) {
    const dim3 grid((S.N + kBlock - 1) / kBlock), block(kBlock);
    if (h->cfg.mode == USV_MODE_ASMC_V0)
      hipLaunchKernelGGL((v0_step_kernel<R>), grid, block, 0, st, S, io);
    else if (h->cfg.mode == USV_MODE_ASMC_YE_INT_V0)
      hipLaunchKernelGGL((legacy_step_kernel<R, kFamYeInt>), grid, block, 0, st, S, io);
    else
      hipLaunchKernelGGL((legacy_step_kernel<R, kFamPid>), grid, block, 0, st, S, io);
    HIP_TRY(hipGetLastError());
    return USV_OK;
  }
  const int epb = h->epb, lid = h->lid;
  const bool simple = h->cfg.mode == USV_MODE_SIMPLE;
  void* args[] = {(void*)&S, (void*)&io};
  if constexpr (std::is_same<R, float>::value) {
    if (h->kind == 4 || h->kind == 5 || h->kind == 6) {     // block-queue step, kQE envs per block
      if (h->kind == 4) {
        void* dyn = simple ? (void*)&dyn_rec_kernel<USV_MODE_SIMPLE> : (void*)&dyn_rec_kernel<USV_MODE_ASMC_SIMPLE>;
        HIP_TRY(hipLaunchKernel(dyn, dim3((S.N + kBlock - 1) / kBlock), dim3(kBlock), args, 0, st));
      }
      if (h->kind == 6)                                      // usv-asmc-simple: the ASMC chain first
        HIP_TRY(hipLaunchKernel((void*)&asmc_chain_kernel<float>, dim3((S.N + kBlock - 1) / kBlock), dim3(kBlock), args, 0, st));
      const bool small = h->kind != 4 && h->epb == kQE_S;
      const int qe = small ? kQE_S : kQE, qw = small ? kQW_S : kQW;
      // a one-round grid of the 128-env blocks: the second block of each CU raises priority
      const int nblk = (S.N + qe - 1) / qe;
      S.qyoung = (!small && nblk > h->cus && nblk <= 2 * h->cus) ? h->cus : INT_MAX;
      HIP_TRY(hipLaunchKernel(pick_q(h->cfg.mode, h->kind != 4, small, io.done != nullptr, h->kind == 6,
                                     io.info != nullptr, S.rowspan != 0),
                              dim3((S.N + qe - 1) / qe), dim3(qw * kWave), args,
                              small ? lds_q_bytes<kQE_S, kQW_S>() : lds_q_bytes(), st));
      return USV_OK;
    }
  }
  if constexpr (std::is_same<R, double>::value) {
    if (h->kind == 3) {                                     // fused, block-wide dynamics (f64 usv-simple)
      void* fn = epb == 64 ? (void*)&step_kernel_blockdyn<R, USV_MODE_SIMPLE, 16, 7>
                           : (void*)&step_kernel_blockdyn<R, USV_MODE_SIMPLE, 8, 7>;
      HIP_TRY(hipLaunchKernel(fn, dim3((S.N + epb - 1) / epb), dim3(kBlock), args, lds_blockdyn_bytes<R>(S.cap), st));
      return USV_OK;
    }
  }
  if (h->kind == 2) {                                       // split: dynamics, then the wave scan
    void* dyn = simple ? (void*)&dyn_kernel<R, USV_MODE_SIMPLE> : (void*)&dyn_kernel<R, USV_MODE_ASMC_SIMPLE>;
    HIP_TRY(hipLaunchKernel(dyn, dim3((S.N + kBlock - 1) / kBlock), dim3(kBlock), args, 0, st));
    void* fn = simple ? pick_scan<R, USV_MODE_SIMPLE, kWaves>(epb / kWaves, lid)
                      : pick_scan<R, USV_MODE_ASMC_SIMPLE, kWaves>(epb / kWaves, lid);
    HIP_TRY(hipLaunchKernel(fn, dim3((S.N + epb - 1) / epb), dim3(kBlock), args, lds_scan_bytes<R>(S.cap), st));
    return USV_OK;
  }
  size_t lds;                                               // kind 1: fused wave kernel
  void* fn = simple ? pick_wave<R, USV_MODE_SIMPLE>(epb / kWaves, lid, &lds, S.cap)
                    : pick_wave<R, USV_MODE_ASMC_SIMPLE>(epb / kWaves, lid, &lds, S.cap);
  HIP_TRY(hipLaunchKernel(fn, dim3((S.N + epb - 1) / epb), dim3(kBlock), args, lds, st));
  return USV_OK;
}

template <typename R>
int launch_reset(Handle* h, State<R>& S, const uint8_t* mask, float* obs, int kpath, void* info,
                 hipStream_t st) {
  IO<R> io{nullptr, obs, nullptr, nullptr, nullptr, nullptr, mask, is_legacy(h->cfg.mode) ? nullptr : (R*)info, kpath};
  const dim3 grid((S.N + kEPBReset - 1) / kEPBReset), block(kBlock);
  const dim3 lgrid((S.N + kBlock - 1) / kBlock);
  if (h->cfg.mode == USV_MODE_ASMC_V0)
    hipLaunchKernelGGL((v0_reset_kernel<R, kFamV0>), lgrid, block, 0, st, S, io);
  else if (h->cfg.mode == USV_MODE_ASMC_YE_INT_V0)
    hipLaunchKernelGGL((v0_reset_kernel<R, kFamYeInt>), lgrid, block, 0, st, S, io);
  else if (h->cfg.mode == USV_MODE_PID_V0)
    hipLaunchKernelGGL((v0_reset_kernel<R, kFamPid>), lgrid, block, 0, st, S, io);
  else if (h->cfg.mode == USV_MODE_SIMPLE)
    hipLaunchKernelGGL((reset_kernel<R, USV_MODE_SIMPLE>), grid, block, lds_head_bytes<R>() + kWaves * 3 * 64 * sizeof(R), st, S, io);
  else
    hipLaunchKernelGGL((reset_kernel<R, USV_MODE_ASMC_SIMPLE>), grid, block, lds_head_bytes<R>() + kWaves * 3 * 64 * sizeof(R), st, S, io);
  HIP_TRY(hipGetLastError());
  return USV_OK;
}

int field_per_env(const Handle* h, int f) {
  if (f >= USV_FIELD_OBS_X && f <= USV_FIELD_OBS_R) return h->cfg.obstacle_cap;
  if (f == USV_FIELD_SENSOR_LAST) return kSensors;
  if (f == USV_FIELD_ASMC) return kAsmcN;
  if (f == USV_FIELD_V0_LAST) return 9;
  if (f == USV_FIELD_V0_AUX) return 3;
  if (f == USV_FIELD_V0_TARGET) return 6;
  if (f == USV_FIELD_V0_YE) return 2;
  if (f == USV_FIELD_NP_RNG) return 10;
  if (f == USV_FIELD_NP_MT) return is_legacy(h->cfg.mode) ? 625 : 0;
  return 1;
}

// first v0 SoA row of a v0 field
int v0_base(int f) {
  return f == USV_FIELD_V0_LAST ? kV0Last : f == USV_FIELD_V0_AUX ? kV0Aux
       : f == USV_FIELD_V0_TARGET ? kV0Target : f == USV_FIELD_V0_YE ? kV0Ye : kV0ALast;
}

// host <-> device for one field; host side [N][per] float64 / int32
template <typename R>
int field_io_impl(Handle* h, State<R>& S, int f, void* host, bool to_host);
// Writes complete before returning (hipMemcpy from pageable memory may return before the DMA
// lands), so a kernel the caller launches next on any stream sees them.
template <typename R>
int field_io(Handle* h, State<R>& S, int f, void* host, bool to_host) {
  HIP_TRY(hipDeviceSynchronize());
  const int rc = field_io_impl(h, S, f, host, to_host);
  if (rc == USV_OK && !to_host) HIP_TRY(hipDeviceSynchronize());
  return rc;
}
// f32 usv-simple / usv-asmc-simple keep the heading as phi + 2 pi k (store_heading): the host sees
// and sets the reference's heading, and UsvAsmc's psi_d_last in the reference's frame.
template <typename R>
bool turn_frame(const Handle* h) {
  return std::is_same<R, float>::value && !is_legacy(h->cfg.mode);
}
template <typename R>
int heading_io(Handle* h, State<R>& S, int f, double* hd, bool to_host) {
  const size_t N = (size_t)S.N;
  constexpr double kTwoPi = 2.0 * kPi;
  std::vector<int32_t> k(N);
  HIP_TRY(hipMemcpy(k.data(), S.I(I_TURNS), N * 4, hipMemcpyDeviceToHost));
  std::vector<R> t(N);
  R* dev = f == USV_FIELD_PSI ? S.F(F_PSI) : S.asmc;          // ASMC row 0: psi_d_last
  if (to_host) {
    HIP_TRY(hipMemcpy(t.data(), dev, N * sizeof(R), hipMemcpyDeviceToHost));
    for (size_t e = 0; e < N; ++e) {
      const double v = (double)t[e] + kTwoPi * k[e];
      if (f == USV_FIELD_PSI) hd[e] = v;
      else hd[e * kAsmcN] = v;
    }
    return USV_OK;
  }
  if (f == USV_FIELD_ASMC) {
    HIP_TRY(hipMemcpy(t.data(), dev, N * sizeof(R), hipMemcpyDeviceToHost));   // (rows 1.. already written)
    for (size_t e = 0; e < N; ++e) t[e] = (R)(hd[e * kAsmcN] - kTwoPi * k[e]);
    HIP_TRY(hipMemcpy(dev, t.data(), N * sizeof(R), hipMemcpyHostToDevice));
    return USV_OK;
  }
  // a new heading: new whole turns, and usv-asmc-simple's psi_d_last moved into the new frame.
  // The turn count is an int32: a non-finite heading, or one whose turns do not fit (|psi| beyond
  // about 1.3e10 rad), is refused before anything is written.
  for (size_t e = 0; e < N; ++e)
    if (!std::isfinite(hd[e]) || std::fabs(hd[e] / kTwoPi) > 2147483000.0)
      return fail(USV_ERR_ARG, "heading must be finite with |psi| / 2 pi < 2^31");
  std::vector<int32_t> kn(N);
  for (size_t e = 0; e < N; ++e) {
    const double n = std::nearbyint(hd[e] / kTwoPi);
    kn[e] = (int32_t)n;
    t[e] = (R)(hd[e] - kTwoPi * n);
  }
  HIP_TRY(hipMemcpy(dev, t.data(), N * sizeof(R), hipMemcpyHostToDevice));
  if (h->cfg.mode == USV_MODE_ASMC_SIMPLE) {
    std::vector<R> s0(N);
    HIP_TRY(hipMemcpy(s0.data(), S.asmc, N * sizeof(R), hipMemcpyDeviceToHost));
    for (size_t e = 0; e < N; ++e) s0[e] = (R)((double)s0[e] + kTwoPi * (k[e] - kn[e]));
    HIP_TRY(hipMemcpy(S.asmc, s0.data(), N * sizeof(R), hipMemcpyHostToDevice));
  }
  HIP_TRY(hipMemcpy(S.I(I_TURNS), kn.data(), N * 4, hipMemcpyHostToDevice));
  return USV_OK;
}

template <typename R>
int field_io_impl(Handle* h, State<R>& S, int f, void* host, bool to_host) {
  const size_t N = (size_t)S.N;
  if (f == USV_FIELD_PSI && turn_frame<R>(h)) return heading_io<R>(h, S, f, (double*)host, to_host);
  if (f < F_NREAL) {
    std::vector<R> tmp(N);
    double* hd = (double*)host;
    if (to_host) {
      HIP_TRY(hipMemcpy(tmp.data(), S.F(f), N * sizeof(R), hipMemcpyDeviceToHost));
      for (size_t i = 0; i < N; ++i) hd[i] = (double)tmp[i];
    } else {
      for (size_t i = 0; i < N; ++i) tmp[i] = (R)hd[i];
      HIP_TRY(hipMemcpy(S.F(f), tmp.data(), N * sizeof(R), hipMemcpyHostToDevice));
    }
    return USV_OK;
  }
  if (f >= USV_FIELD_N_OBS && f <= USV_FIELD_SCAN_VALID) {
    int32_t* d = S.I(f - USV_FIELD_N_OBS);
    if (!to_host && f == USV_FIELD_N_OBS) {
      const int32_t* hv = (const int32_t*)host;
      for (size_t i = 0; i < N; ++i)
        if (hv[i] < 0 || hv[i] > S.cap) return fail(USV_ERR_ARG, "n_obs out of [0, obstacle_cap]");
    }
    if (to_host) HIP_TRY(hipMemcpy(host, d, N * 4, hipMemcpyDeviceToHost));
    else HIP_TRY(hipMemcpy(d, host, N * 4, hipMemcpyHostToDevice));
    return USV_OK;
  }
  if (f >= USV_FIELD_OBS_X && f <= USV_FIELD_OBS_R) {   // device [N][3][ostride], host [N][cap]
    const size_t os = (size_t)S.ostride, cnt = N * 3 * os, cap = (size_t)S.cap;
    std::vector<R> tmp(cnt);
    HIP_TRY(hipMemcpy(tmp.data(), S.obst, cnt * sizeof(R), hipMemcpyDeviceToHost));
    double* hd = (double*)host;
    const size_t plane = (size_t)(f - USV_FIELD_OBS_X);   // x / y / r
    for (size_t e = 0; e < N; ++e)
      for (size_t j = 0; j < cap; ++j) {
        R& v = tmp[(e * 3 + plane) * os + j];
        if (to_host) hd[e * cap + j] = (double)v;
        else v = (R)hd[e * cap + j];
      }
    if (!to_host) HIP_TRY(hipMemcpy(S.obst, tmp.data(), cnt * sizeof(R), hipMemcpyHostToDevice));
    return USV_OK;
  }
  if (f == USV_FIELD_SENSOR_LAST) {
    const size_t cnt = N * kSensors;
    std::vector<R> tmp(cnt);
    double* hd = (double*)host;
    if (to_host) {
      HIP_TRY(hipMemcpy(tmp.data(), S.sensor_last, cnt * sizeof(R), hipMemcpyDeviceToHost));
      for (size_t i = 0; i < cnt; ++i) hd[i] = (double)tmp[i];
    } else {
      for (size_t i = 0; i < cnt; ++i) tmp[i] = (R)hd[i];
      HIP_TRY(hipMemcpy(S.sensor_last, tmp.data(), cnt * sizeof(R), hipMemcpyHostToDevice));
    }
    return USV_OK;
  }
  if (f == USV_FIELD_ASMC) {   // device [16][N], host [N][16]
    const size_t cnt = N * kAsmcN;
    std::vector<R> tmp(cnt);
    double* hd = (double*)host;
    if (to_host) {
      HIP_TRY(hipMemcpy(tmp.data(), S.asmc, cnt * sizeof(R), hipMemcpyDeviceToHost));
      for (size_t e = 0; e < N; ++e)
        for (int i = 0; i < kAsmcN; ++i) hd[e * kAsmcN + i] = (double)tmp[(size_t)i * N + e];
    } else {
      for (size_t e = 0; e < N; ++e)
        for (int i = 0; i < kAsmcN; ++i) tmp[(size_t)i * N + e] = (R)hd[e * kAsmcN + i];
      HIP_TRY(hipMemcpy(S.asmc, tmp.data(), cnt * sizeof(R), hipMemcpyHostToDevice));
    }
    // psi_d_last between the reference's frame (host) and the heading's (device, f32)
    if (turn_frame<R>(h)) return heading_io<R>(h, S, f, hd, to_host);
    return USV_OK;
  }
  if (f == USV_FIELD_NP_RNG || f == USV_FIELD_NP_MT) {   // device SoA uint32 rows, host [N][per] int32
    const int per = field_per_env(h, f);
    std::vector<uint32_t> tmp(N);
    uint32_t* hd = (uint32_t*)host;
    for (int i = 0; i < per; ++i) {
      uint32_t* d = (f == USV_FIELD_NP_RNG ? S.nprng : S.npmt) + (size_t)i * S.fstride;
      if (to_host) {
        HIP_TRY(hipMemcpy(tmp.data(), d, N * 4, hipMemcpyDeviceToHost));
        for (size_t e = 0; e < N; ++e) hd[e * per + i] = tmp[e];
      } else {
        for (size_t e = 0; e < N; ++e) tmp[e] = hd[e * per + i];
        HIP_TRY(hipMemcpy(d, tmp.data(), N * 4, hipMemcpyHostToDevice));
      }
    }
    return USV_OK;
  }
  if (f >= USV_FIELD_V0_LAST && f <= USV_FIELD_V0_YE) {   // device SoA rows, host [N][per]
    const int per = field_per_env(h, f), base = v0_base(f);
    std::vector<R> tmp(N);
    double* hd = (double*)host;
    for (int i = 0; i < per; ++i) {
      if (to_host) {
        HIP_TRY(hipMemcpy(tmp.data(), S.V(base + i), N * sizeof(R), hipMemcpyDeviceToHost));
        for (size_t e = 0; e < N; ++e) hd[e * per + i] = (double)tmp[e];
      } else {
        for (size_t e = 0; e < N; ++e) tmp[e] = (R)hd[e * per + i];
        HIP_TRY(hipMemcpy(S.V(base + i), tmp.data(), N * sizeof(R), hipMemcpyHostToDevice));
      }
    }
    return USV_OK;
  }
  return fail(USV_ERR_ARG, "unknown field");
}

size_t field_bytes(const Handle* h, int f) {
  return (size_t)h->cfg.num_envs * field_per_env(h, f) * (kFields[f].is_int ? 4 : 8);
}

template <typename R>
int set_experiment(Handle* h, State<R>& S, const usv_experiment* x) {
  HIP_TRY(hipDeviceSynchronize());                       // in-flight resets may read the old one
  if (!x) {
    S.exp = nullptr;
    return USV_OK;
  }
  const int cap = h->cfg.obstacle_cap;
  std::vector<R> v((size_t)kExpObs + 3 * cap, R(0));
  v[kExpN] = (R)x->n_obs;
  v[kExpPS] = (R)x->path_start[0]; v[kExpPS + 1] = (R)x->path_start[1];
  v[kExpAngle] = (R)x->angle;
  for (int i = 0; i < 3; ++i) v[kExpPose + i] = (R)x->position[i];
  for (int j = 0; j < x->n_obs; ++j) {
    v[kExpObs + j] = (R)x->obstacle_x[j];
    v[kExpObs + cap + j] = (R)x->obstacle_y[j];
    v[kExpObs + 2 * cap + j] = (R)x->obstacle_r[j];
  }
  HIP_TRY(hipMemcpy(h->exp_buf, v.data(), v.size() * sizeof(R), hipMemcpyHostToDevice));
  HIP_TRY(hipDeviceSynchronize());
  S.exp = (const R*)h->exp_buf;
  return USV_OK;
}

// The block-queue step's LDS exceeds the 64 KiB default: raise the kernels' dynamic-LDS limit.
int queue_lds_attr(const Handle* h) {
  if (h->kind != 4 && h->kind != 5 && h->kind != 6) return USV_OK;
  const bool split = h->kind == 6;
  for (const bool done : {false, true})
    for (const bool info : {false, true}) {
      for (const bool span : {false, true})
        HIP_TRY(hipFuncSetAttribute(pick_q(h->cfg.mode, h->kind != 4, false, done, split, info, span),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_q_bytes()));
      if (h->kind != 4)
        HIP_TRY(hipFuncSetAttribute(pick_q(h->cfg.mode, true, true, done, split, info),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_q_bytes<kQE_S, kQW_S>()));
    }
  return USV_OK;
}

Handle* as_handle(void* p) { return static_cast<Handle*>(p); }

}  // namespace

extern "C" {

int usv_abi_version(void) { return USV_ABI_VERSION; }

#ifdef USV_DIAG_PROF
int usv_diag_prof(void* host, size_t bytes) {
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_prof), bytes < sizeof(g_prof) ? bytes : sizeof(g_prof)));
  return USV_OK;
}
#endif
#ifdef USV_DIAG_QPROF
int usv_diag_qprof(void* host, size_t bytes) {
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_qprof), bytes < sizeof(g_qprof) ? bytes : sizeof(g_qprof)));
  return USV_OK;
}
#endif
#ifdef USV_DIAG_STAMPS
int usv_diag_stamps(void* host, size_t bytes) {
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), bytes < sizeof(g_stamps) ? bytes : sizeof(g_stamps)));
  return USV_OK;
}
#endif

const char* usv_last_error(void) { return g_err.c_str(); }

size_t usv_config_size(void) { return sizeof(usv_config); }

int usv_asmc_compute(int32_t precision, int32_t n, const void* act, void* pos, void* vel, void* state,
                     int32_t* perturb_step, int32_t do_perturb, int32_t calls, void* stream) {
  if (precision != USV_F32 && precision != USV_F64) return fail(USV_ERR_ARG, "unknown precision");
  if (n < 0 || calls < 0) return fail(USV_ERR_ARG, "n and calls must be >= 0");
  if (n == 0 || calls == 0) return USV_OK;
  if (!act || !pos || !vel || !state) return fail(USV_ERR_ARG, "null argument");
  // launch on the device that holds the state, whatever the caller's current device is; every buffer
  // must be device-accessible memory of that device (a pageable host pointer would fault the kernel)
  auto device_of = [](const void* p) {
    hipPointerAttribute_t pa{};
    return hipPointerGetAttributes(&pa, p) == hipSuccess ? pa.device : -1;
  };
  const int dev = device_of(state);
  if (dev < 0) { (void)hipGetLastError(); return fail(USV_ERR_ARG, "state is not a device pointer"); }
  if (device_of(act) != dev || device_of(pos) != dev || device_of(vel) != dev ||
      (perturb_step && device_of(perturb_step) != dev)) {
    (void)hipGetLastError();
    return fail(USV_ERR_ARG, "act / pos / vel / perturb_step are not device pointers on the state's device");
  }
  DeviceGuard g(dev);
  const dim3 grid((n + kBlock - 1) / kBlock), block(kBlock);
  hipStream_t st = (hipStream_t)stream;
  if (precision == USV_F32)
    hipLaunchKernelGGL(asmc_compute_kernel<float>, grid, block, 0, st, n, (const float*)act, (float*)pos,
                       (float*)vel, (float*)state, perturb_step, do_perturb, calls);
  else
    hipLaunchKernelGGL(asmc_compute_kernel<double>, grid, block, 0, st, n, (const double*)act, (double*)pos,
                       (double*)vel, (double*)state, perturb_step, do_perturb, calls);
  HIP_TRY(hipGetLastError());
  return USV_OK;
}

void usv_config_default(usv_config* cfg, int32_t mode, int32_t num_envs) {
  if (!cfg) return;
  std::memset(cfg, 0, sizeof(*cfg));
  cfg->abi_version = USV_ABI_VERSION;
  cfg->mode = mode;
  cfg->precision = USV_F32;
  cfg->num_envs = num_envs;
  cfg->obstacle_cap = 32;
  cfg->max_episode_steps = mode == USV_MODE_ASMC_SIMPLE ? 1000 : is_legacy(mode) ? 0 : 500;  // gym_usv/__init__.py
  cfg->autoreset = USV_AUTORESET_SAME_STEP;
  cfg->lidar_algo = USV_LIDAR_WINDOW;
  cfg->seed = 0;
  cfg->env_id_offset = 0;
}

int usv_create(const usv_config* cfg, int32_t device, void** out) {
  if (!cfg || !out) return fail(USV_ERR_ARG, "null argument");
  *out = nullptr;
  if (cfg->abi_version != USV_ABI_VERSION) return fail(USV_ERR_ABI, "abi_version mismatch");
  if (cfg->mode != USV_MODE_SIMPLE && cfg->mode != USV_MODE_ASMC_SIMPLE && !is_legacy(cfg->mode))
    return fail(USV_ERR_ARG, "unknown mode");
  if (cfg->precision != USV_F32 && cfg->precision != USV_F64)
    return fail(USV_ERR_ARG, "unknown precision");
  if (cfg->num_envs <= 0) return fail(USV_ERR_ARG, "num_envs must be > 0");
  if (cfg->obstacle_cap < 29 || cfg->obstacle_cap > 64)
    return fail(USV_ERR_ARG, "obstacle_cap must be in [29, 64] (reference draws up to 29)");
  if (cfg->autoreset != USV_AUTORESET_SAME_STEP && cfg->autoreset != USV_AUTORESET_DISABLED)
    return fail(USV_ERR_ARG, "unknown autoreset mode");
  if (cfg->lidar_algo != USV_LIDAR_BRUTE && cfg->lidar_algo != USV_LIDAR_WINDOW)
    return fail(USV_ERR_ARG, "unknown lidar algorithm");
  if ((cfg->flags & ~USV_FLAG_PERTURB) != 0 || cfg->reserved != 0) return fail(USV_ERR_ARG, "unknown flags");
  if ((cfg->flags & USV_FLAG_PERTURB) && cfg->mode != USV_MODE_ASMC_SIMPLE)
    return fail(USV_ERR_ARG, "USV_FLAG_PERTURB applies to usv-asmc-simple only");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(USV_ERR_ARG, "bad device index");
  DeviceGuard g(device);
  Handle* h = new Handle();
  h->cfg = *cfg;
  h->device = device;
  {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
      h->cus = cus;
  }
  h->lid = cfg->lidar_algo == USV_LIDAR_BRUTE ? (kLidSkip | kLidUnroll2) : (kLidSkip | kLidUnroll2 | kLidWindow);
  // tuned defaults at 65 536 envs on MI355X (tools/sweep_variants.py, profiles/): usv-simple
  // (f32, window lidar) runs the fused block-queue step, else the fused wave kernel at 16
  // envs/wave; usv-asmc-simple the split block-queue step, else the split wave scan at 4 envs/wave
  const bool queue = cfg->precision == USV_F32 && cfg->lidar_algo == USV_LIDAR_WINDOW && cfg->obstacle_cap <= 32;
  if (cfg->mode == USV_MODE_ASMC_SIMPLE) {
    // ASMC's 20 substeps want full-width dynamics: a separate dyn_kernel, then the block queue
    // (45.7 us vs 46.7 for the split wave scan at 65 536 envs)
    // f64 (window lidar, cap <= 32): the split f64 wave scan at 16 envs/wave from 49 152 envs
    // (72.0 us at 65 536 envs against 77.4 at 4); block-wide dynamics (kind 3) spill the f64 ASMC
    // state at 4 waves per SIMD (94 us)
    const bool f64w = cfg->precision == USV_F64 && cfg->lidar_algo == USV_LIDAR_WINDOW && cfg->obstacle_cap <= 32;
    // f32 (window lidar, cap <= 32): the ASMC chain in its own launch, then the fused block-queue step
    // with usv-simple's phase 1 (kind 6), small blocks below kQSmallBelow envs
    if (queue) { h->kind = 6; h->epb = cfg->num_envs < kQSmallBelow ? kQE_S : kQE; }
    else if (f64w) { h->kind = 2; h->epb = cfg->num_envs >= 49152 ? 64 : 32; }
    else { h->kind = 2; h->epb = 16; }
  } else if (queue) {
    h->kind = 5;                        // block-queue step: 16-wave blocks of 128 envs, or 8-wave blocks
    h->epb = cfg->num_envs < kQSmallBelow ? kQE_S : kQE;   // of 16 below kQSmallBelow envs
  } else if (cfg->precision == USV_F64 && cfg->lidar_algo == USV_LIDAR_WINDOW && cfg->obstacle_cap <= 32) {
    // f64: one launch, wave 0 of each block runs the block's dynamics at full width, then the
    // two-env wave scan (kind 3); 16 envs/wave from 49 152 envs up (one round of 4 waves per SIMD
    // at 65 536 envs: 40.3 us, against 47.7 for the split dyn_kernel + scan), else 8
    h->kind = 3; h->epb = cfg->num_envs >= 49152 ? 64 : 32;
  } else { h->kind = 1; h->epb = 64; }
  h->prio = h->kind >= 4 ? 0 : kStaticPrio;   // the ramp helps static splits only
  if (const int rc = queue_lds_attr(h); rc != USV_OK) { delete h; return rc; }
  const int rc = cfg->precision == USV_F32 ? carve<float>(h, h->sf) : carve<double>(h, h->sd);
  if (rc != USV_OK) {
    if (h->slab) (void)hipFree(h->slab);
    delete h;
    return rc;
  }
  *out = h;
  return USV_OK;
}

int usv_set_kernel_variant(void* hp, int32_t kind, int32_t epb, int32_t lid) {
  Handle* h = as_handle(hp);
  if (!h) return fail(USV_ERR_ARG, "null handle");
  if (is_legacy(h->cfg.mode)) return fail(USV_ERR_ARG, "the legacy ids have one lane-per-env kernel");
  const usv_config* cfg = &h->cfg;
  // lid bits 0x100 / 0x200: the block-queue step's row-span stores forced on / off (State::rowspan)
  const int rs = lid & 0x300;
  lid &= 0xff;
  if (rs == 0x300 || (rs && kind != 4 && kind != 5 && kind != 6)) return fail(USV_ERR_ARG, "bad row-store bits");
  const bool lid_ok = lid == 0 || lid == 3 || lid == 7;
  const bool wave_ok = kind == 1 && (epb == 16 || epb == 32 || epb == 64) && lid_ok;
  const bool split_ok = kind == 2 && (epb == 8 || epb == 16 || epb == 32 ||
                                      (epb == 64 && lid == 7 && cfg->precision == USV_F64)) && lid_ok;
  const bool blockdyn_ok = kind == 3 && (epb == 32 || epb == 64) && lid == 7 && cfg->precision == USV_F64 &&
                           cfg->mode == USV_MODE_SIMPLE;
  const bool queue_ok = (kind == 4 || kind == 5 || (kind == 6 && cfg->mode == USV_MODE_ASMC_SIMPLE)) &&
                        (epb == kQE || (kind != 4 && epb == kQE_S)) && lid == 7 &&
                        cfg->precision == USV_F32 && cfg->obstacle_cap <= 32;
  if (!(wave_ok || split_ok || blockdyn_ok || queue_ok)) return fail(USV_ERR_ARG, "kernel variant not available for this config");
  DeviceGuard g(h->device);
  HIP_TRY(hipDeviceSynchronize());                 // launches in flight keep the variant they took
  Handle trial = *h;                               // raise the new variant's LDS limit first, and
  trial.kind = kind;                               // commit it to the handle only if that worked
  trial.epb = epb;
  if (const int rc = queue_lds_attr(&trial); rc != USV_OK) return rc;
  h->kind = kind;
  h->epb = epb;
  h->lid = lid;
  h->prio = kind >= 4 ? 0 : kStaticPrio;
  h->sf.prio = h->sd.prio = h->prio;
  h->sf.rowspan = h->sd.rowspan = rs ? rs == 0x100 : h->cfg.num_envs >= kRowSpanFrom;
  return USV_OK;
}

void usv_destroy(void* hp) {
  Handle* h = as_handle(hp);
  if (!h) return;
  DeviceGuard g(h->device);
  (void)hipDeviceSynchronize();
  if (h->slab) (void)hipFree(h->slab);
  delete h;
}

int usv_num_envs(void* hp) { return hp ? as_handle(hp)->cfg.num_envs : fail(USV_ERR_ARG, "null handle"); }
int usv_obs_dim(void* hp) {
  return hp ? (is_legacy(as_handle(hp)->cfg.mode) ? 6 : kObsDim) : fail(USV_ERR_ARG, "null handle");
}
int usv_act_dim(void* hp) {
  return hp ? (is_legacy(as_handle(hp)->cfg.mode) ? 1 : 2) : fail(USV_ERR_ARG, "null handle");
}
int usv_reward_bytes(void* hp) {
  return hp ? (as_handle(hp)->cfg.precision == USV_F64 ? 8 : 4) : fail(USV_ERR_ARG, "null handle");
}

int usv_set_reset_rng(void* hp, int32_t kind) {
  Handle* h = as_handle(hp);
  if (!h) return fail(USV_ERR_ARG, "null handle");
  if (kind != USV_RESET_PHILOX && kind != USV_RESET_NUMPY_PCG64) return fail(USV_ERR_ARG, "unknown reset rng");
  h->sf.np_reset = h->sd.np_reset = kind == USV_RESET_NUMPY_PCG64;
  return USV_OK;
}

int usv_seed(void* hp, uint64_t seed) {
  Handle* h = as_handle(hp);
  if (!h) return fail(USV_ERR_ARG, "null handle");
  DeviceGuard g(h->device);
  h->cfg.seed = seed;
  h->sf.seed = seed;
  h->sd.seed = seed;
  int32_t* ep = h->cfg.precision == USV_F32 ? h->sf.I(I_EPISODE) : h->sd.I(I_EPISODE);
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemset(ep, 0, (size_t)h->cfg.num_envs * 4));
  HIP_TRY(hipDeviceSynchronize());     // ordered before launches on any (non-blocking) stream
  return USV_OK;
}

int usv_reset_ex(void* hp, const uint8_t* mask, float* obs, const usv_reset_options* opt, void* info,
                 void* stream) {
  Handle* h = as_handle(hp);
  if (!h || !obs) return fail(USV_ERR_ARG, "null argument");
  const int kpath = opt ? opt->place_obstacles_on_path : 0;
  if (kpath < 0) return fail(USV_ERR_ARG, "place_obstacles_on_path must be >= 0");
  if (kpath > 0 && is_legacy(h->cfg.mode))
    return fail(USV_ERR_ARG, "place_obstacles_on_path applies to usv-simple / usv-asmc-simple only");
  if (kpath > 0 && 29 + kpath > h->cfg.obstacle_cap)
    return fail(USV_ERR_ARG, "place_obstacles_on_path needs obstacle_cap >= 29 + k (reference draws up to 29)");
  DeviceGuard g(h->device);
  hipStream_t st = (hipStream_t)stream;
  return h->cfg.precision == USV_F32 ? launch_reset<float>(h, h->sf, mask, obs, kpath, info, st)
                                     : launch_reset<double>(h, h->sd, mask, obs, kpath, info, st);
}

int usv_reset(void* hp, const uint8_t* mask, float* obs, void* stream) {
  return usv_reset_ex(hp, mask, obs, nullptr, nullptr, stream);
}

int usv_step_ex(void* hp, const float* act, float* obs, void* rew, uint8_t* term, uint8_t* trunc,
                uint8_t* done, float* fobs, void* info, void* stream) {
  Handle* h = as_handle(hp);
  if (!h || !act || !obs || !rew || !term || !trunc) return fail(USV_ERR_ARG, "null argument");
  DeviceGuard g(h->device);
  hipStream_t st = (hipStream_t)stream;
  return h->cfg.precision == USV_F32
             ? launch_step<float>(h, h->sf, act, obs, rew, term, trunc, done, fobs, info, st)
             : launch_step<double>(h, h->sd, act, obs, rew, term, trunc, done, fobs, info, st);
}

int usv_step(void* hp, const float* act, float* obs, void* rew, uint8_t* term, uint8_t* trunc,
             float* fobs, void* stream) {
  return usv_step_ex(hp, act, obs, rew, term, trunc, nullptr, fobs, nullptr, stream);
}

int usv_set_experiment(void* hp, const usv_experiment* x) {
  Handle* h = as_handle(hp);
  if (!h) return fail(USV_ERR_ARG, "null handle");
  if (is_legacy(h->cfg.mode)) return fail(USV_ERR_ARG, "custom experiments apply to usv-simple / usv-asmc-simple only");
  if (x && (x->n_obs < 1 || x->n_obs > h->cfg.obstacle_cap || x->n_obs > 64))
    return fail(USV_ERR_ARG, "experiment n_obs must be in [1, obstacle_cap]");
  DeviceGuard g(h->device);
  return h->cfg.precision == USV_F32 ? set_experiment<float>(h, h->sf, x) : set_experiment<double>(h, h->sd, x);
}

int usv_field_info(void* hp, int32_t f, int32_t* per_env, int32_t* is_int, const char** name) {
  Handle* h = as_handle(hp);
  if (!h || f < 0 || f >= USV_FIELD_COUNT) return fail(USV_ERR_ARG, "bad handle or field");
  if (per_env) *per_env = field_per_env(h, f);
  if (is_int) *is_int = kFields[f].is_int;
  if (name) *name = kFields[f].name;
  return USV_OK;
}

int usv_get_field(void* hp, int32_t f, void* host, size_t bytes) {
  Handle* h = as_handle(hp);
  if (!h || !host || f < 0 || f >= USV_FIELD_COUNT) return fail(USV_ERR_ARG, "bad argument");
  if (bytes != field_bytes(h, f)) return fail(USV_ERR_ARG, "byte count mismatch");
  DeviceGuard g(h->device);
  return h->cfg.precision == USV_F32 ? field_io<float>(h, h->sf, f, host, true)
                                     : field_io<double>(h, h->sd, f, host, true);
}

int usv_set_field(void* hp, int32_t f, const void* host, size_t bytes) {
  Handle* h = as_handle(hp);
  if (!h || !host || f < 0 || f >= USV_FIELD_COUNT) return fail(USV_ERR_ARG, "bad argument");
  if (bytes != field_bytes(h, f)) return fail(USV_ERR_ARG, "byte count mismatch");
  DeviceGuard g(h->device);
  return h->cfg.precision == USV_F32 ? field_io<float>(h, h->sf, f, (void*)host, false)
                                     : field_io<double>(h, h->sd, f, (void*)host, false);
}

size_t usv_state_bytes(void* hp) {
  Handle* h = as_handle(hp);
  if (!h) return 0;
  size_t b = 0;
  for (int f = 0; f < USV_FIELD_COUNT; ++f) b += field_bytes(h, f);
  return b;
}

int usv_get_state(void* hp, void* host, size_t bytes) {
  Handle* h = as_handle(hp);
  if (!h || !host) return fail(USV_ERR_ARG, "bad argument");
  if (bytes != usv_state_bytes(hp)) return fail(USV_ERR_ARG, "byte count mismatch");
  char* p = (char*)host;
  for (int f = 0; f < USV_FIELD_COUNT; ++f) {
    const size_t fb = field_bytes(h, f);
    const int rc = usv_get_field(hp, f, p, fb);
    if (rc != USV_OK) return rc;
    p += fb;
  }
  return USV_OK;
}

int usv_set_state(void* hp, const void* host, size_t bytes) {
  Handle* h = as_handle(hp);
  if (!h || !host) return fail(USV_ERR_ARG, "bad argument");
  if (bytes != usv_state_bytes(hp)) return fail(USV_ERR_ARG, "byte count mismatch");
  const char* p = (const char*)host;
  for (int f = 0; f < USV_FIELD_COUNT; ++f) {
    const size_t fb = field_bytes(h, f);
    const int rc = usv_set_field(hp, f, p, fb);
    if (rc != USV_OK) return rc;
    p += fb;
  }
  return USV_OK;
}

}  // extern "C"
