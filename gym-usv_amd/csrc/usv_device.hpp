// usv_device.hpp — device-side building blocks of the gfx950 USV step kernels.
//
// Everything here is per-env math written for one of two thread mappings:
//   * lane-per-env  (dynamics, ASMC, reward, reset): struct-of-arrays state, one env per
//                   wavefront lane, coalesced [field][N] loads/stores;
//   * wave-per-env  (lidar + observation row): 64 lanes own 128 rays (2 per lane), the
//                   env's obstacles are wave-uniform and broadcast with v_readlane.
// Reference citations are path:line in romi2002/gym-usv.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

// No implicit a*b+c contraction anywhere in the device code: every fused multiply-add is an
// explicit m_fma/fmaf.  With contraction left to the backend, the same inlined function can
// round differently in different kernels (it depends on the surrounding code), and the step
// kernel variants, the split dynamics kernel and the reset kernel must agree bit for bit.
#pragma clang fp contract(off)

namespace usv {

// ----------------------------------------------------------------------------- constants
constexpr int kSensors = 128;                      // simple_env.py:11
constexpr int kObsDim = 143;                       // simple_env.py:27
constexpr int kHdr = 15;                           // obs[0:15] (simple_env.py:96)
constexpr int kAsmcN = 16;                         // unique UsvAsmc state values
constexpr int kWave = 64;
constexpr double kPi = 3.14159265358979323846;
constexpr double kSensorMax = 100.0;               // simple_env.py:13
constexpr double kDt = 1.0 / 25.0;                 // simple_env.py:35
constexpr double kBound = 20.0;                    // simple_env.py:56
constexpr double kMaxAccU = 1.75, kMaxAccR = 3.0;  // simple_env.py:34
constexpr double kDiag = 28.284271247461902;       // hypot(20, 20), simple_env.py:80
constexpr double kLookahead = (0.005 / 10) * 20;   // simple_env.py:146
constexpr double kTermDist = 0.05;                 // simple_env.py:334
constexpr double kCollDist = 0.2;                  // simple_env.py:155
constexpr double kYeK = 0.075;                     // simple_env.py:166

// UsvAsmc coefficients (usv_asmc.py:7-41)
constexpr double X_U_DOT = -2.25, Y_V_DOT = -23.13, Y_R_DOT = -1.31, N_V_DOT = -16.41,
                 N_R_DOT = -2.79;
constexpr double YVV = -99.99, YVR = -5.49, YRV = -5.49, YRR = -8.8;
constexpr double NVV = -5.49, NVR = -8.8, NRV = -8.8, NRR = -3.49;
constexpr double MASS = 30.0, IZ = 4.1, B_TH = 0.41, C_TH = 0.78;
constexpr double K_U = 0.1, K_PSI = 0.2, KMIN_U = 0.05, KMIN_PSI = 0.2;
constexpr double K2_U = 0.02, K2_PSI = 0.1, MU_U = 0.05, MU_PSI = 0.1;
constexpr double LAMBDA_U = 0.001, LAMBDA_PSI = 1.0;
constexpr double F1 = 2.0, F2 = 2.0, F3 = 2.0;
constexpr double H = 0.01;                         // usv_asmc.py:47
// Yv / Yr / Nv / Nr scale factors (usv_asmc.py:101-108)
constexpr double YV_K = 0.5 * (-40.0 * 1000.0) *
    (1.1 + 0.0045 * (1.01 / 0.09) - 0.1 * (0.27 / 0.09) + 0.016 * ((0.27 / 0.09) * (0.27 / 0.09)));
constexpr double YR_K = 6.0 * (-3.141592 * 1000.0) * 0.09 * 0.09 * 1.01;
constexpr double NV_K = 0.06 * (-3.141592 * 1000.0) * 0.09 * 0.09 * 1.01;
constexpr double NR_K = 0.02 * (-3.141592 * 1000.0) * 0.09 * 0.09 * 1.01 * 1.01;
// M^-1 of M = [[m - Xu', 0, 0], [0, m - Yv', -Yr'], [0, -Nv', Iz - Nr']] (usv_asmc.py:172-174);
// constant, so inverted in closed form here instead of per substep (:226).
constexpr double M00 = MASS - X_U_DOT, M11 = MASS - Y_V_DOT, M12 = -Y_R_DOT, M21 = -N_V_DOT,
                 M22 = IZ - N_R_DOT;
constexpr double MDET = M11 * M22 - M12 * M21;
constexpr double MI00 = 1.0 / M00, MI11 = M22 / MDET, MI12 = -M12 / MDET, MI21 = -M21 / MDET,
                 MI22 = M11 / MDET;

// ----------------------------------------------------------------------------- math shims
__device__ __forceinline__ float  m_sin(float x)  { return sinf(x); }
__device__ __forceinline__ double m_sin(double x) { return sin(x); }
__device__ __forceinline__ float  m_cos(float x)  { return cosf(x); }
__device__ __forceinline__ double m_cos(double x) { return cos(x); }
__device__ __forceinline__ void m_sincos(float x, float* s, float* c) { sincosf(x, s, c); }
__device__ __forceinline__ void m_sincos(double x, double* s, double* c) { sincos(x, s, c); }
__device__ __forceinline__ float  m_atan2(float y, float x)  { return atan2f(y, x); }
__device__ __forceinline__ double m_atan2(double y, double x) { return atan2(y, x); }
__device__ __forceinline__ float  m_asin(float x)  { return asinf(x); }
__device__ __forceinline__ double m_asin(double x) { return asin(x); }
__device__ __forceinline__ float  m_sqrt(float x)  { return sqrtf(x); }
__device__ __forceinline__ double m_sqrt(double x) { return sqrt(x); }
__device__ __forceinline__ float  m_exp(float x)  { return expf(x); }
__device__ __forceinline__ double m_exp(double x) { return exp(x); }
__device__ __forceinline__ float  m_hypot(float x, float y)  { return hypotf(x, y); }
__device__ __forceinline__ double m_hypot(double x, double y) { return hypot(x, y); }
__device__ __forceinline__ float  m_fma(float a, float b, float c)  { return fmaf(a, b, c); }
__device__ __forceinline__ double m_fma(double a, double b, double c) { return fma(a, b, c); }
__device__ __forceinline__ float  m_abs(float x)  { return fabsf(x); }
__device__ __forceinline__ double m_abs(double x) { return fabs(x); }

// Fast paths for the f32 build's per-env scalar math (hardware v_sin/v_cos/v_exp, ~1 ulp at
// the argument ranges here); the f64 build keeps the correctly rounded libm calls.
// The heading psi is unwrapped (simple_env.py:323 integrates it without wrapping), so it is first
// reduced to [-pi, pi] by a two-constant Cody-Waite step: v_sin/v_cos take x / 2pi and lose
// |x| / 2pi * ulp(1) of absolute accuracy in that product, and leave their domain past 256 turns.
__device__ __forceinline__ float reduce_2pi(float x) {
  const float k = rintf(x * 0.159154943f);
  float r = fmaf(-k, 6.28318548f, x);                 // 2 pi rounded to float (high part)
  return fmaf(k, 1.74845553e-07f, r);                 // - k (2 pi - that): the low part is < 0
}
__device__ __forceinline__ void fx_sincos(float x, float* s, float* c) {
  const float r = reduce_2pi(x);
  *s = __sinf(r); *c = __cosf(r);
}
__device__ __forceinline__ void fx_sincos(double x, double* s, double* c) { sincos(x, s, c); }
__device__ __forceinline__ float  fx_exp(float x)  { return __expf(x); }
// atan2 for the f32 step's angle to target: octant reduction with a reciprocal quotient and a degree-15
// odd minimax polynomial (|err| <= 1.4e-7 rad on [0, 1] evaluated in float, ~1 ulp of pi after the
// octant fold): ~20 VALU instead of libm's branchy atan2f on the phase-1 critical path.  The f64
// build keeps libm.
__device__ __forceinline__ float fx_atan2(float y, float x) {
  const float ax = fabsf(x), ay = fabsf(y);
  const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
  const float t = mx > 0.0f ? mn * __builtin_amdgcn_rcpf(mx) : 0.0f;   // hardware reciprocal, 1 ulp
  const float s = t * t;
  float p = -0.004054558929055929f;
  p = fmaf(p, s, 0.021862929686903954f);
  p = fmaf(p, s, -0.055912286043167114f);
  p = fmaf(p, s, 0.09642194956541061f);
  p = fmaf(p, s, -0.1390862911939621f);
  p = fmaf(p, s, 0.19946566224098206f);
  p = fmaf(p, s, -0.33329859375953674f);
  p = fmaf(p, s, 0.9999993443489075f);
  p = p * t;
  p = ay > ax ? 1.57079637f - p : p;
  p = x < 0.0f ? 3.14159274f - p : p;
  return copysignf(p, y);
}
__device__ __forceinline__ double fx_atan2(double y, double x) { return atan2(y, x); }
__device__ __forceinline__ double fx_exp(double x) { return exp(x); }
// x / c for a compile-time constant c: a multiply by the rounded reciprocal in f32 (<= 1 ulp
// apart from the IEEE quotient), the IEEE division in f64
__device__ __forceinline__ float  fx_cdiv(float x, double c)  { return x * (float)(1.0 / c); }
// x / c for a compile-time constant c in double, correctly rounded like the IEEE division it replaces:
// q = RN(x y) with y = RN(1 / c) (folded at compile time) is within one ulp of x / c, r = x - q c is exact
// with one fma, and RN(q + r y) is then x / c correctly rounded (Markstein's theorem; normal operands,
// no overflow).  Three dependent VALU operations instead of the ~10 of a full f64 division; checked
// against x / c on 2e8 random operands for every constant used (0 mismatches).
__device__ __forceinline__ double div_const(double x, double c) {
  const double y = 1.0 / c;
  const double q = x * y;
  return fma(fma(-q, c, x), y, q);
}
__device__ __forceinline__ double fx_cdiv(double x, double c) { return div_const(x, c); }
// a / b via the hardware reciprocal (1 ulp) in f32; IEEE in f64
__device__ __forceinline__ float  fx_div(float a, float b)  { return a * __builtin_amdgcn_rcpf(b); }
__device__ __forceinline__ double fx_div(double a, double b) { return a / b; }
// hardware square root (1 ulp) in f32; IEEE in f64
__device__ __forceinline__ float  fx_sqrt(float x)  { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ double fx_sqrt(double x) { return sqrt(x); }

template <typename T> __device__ __forceinline__ T m_clip(T x, T lo, T hi) {
  // np.clip(x, lo, hi) == minimum(maximum(x, lo), hi)
  x = x > lo ? x : lo;
  return x < hi ? x : hi;
}
template <typename T> __device__ __forceinline__ T m_sign(T x) {   // np.sign: sign(0) = 0
  return x > T(0) ? T(1) : (x < T(0) ? T(-1) : T(0));
}
template <typename T> __device__ __forceinline__ T wrap_once(T e) {  // usv_asmc.py:120
  return m_abs(e) > T(kPi) ? m_sign(e) * (m_abs(e) - T(2 * kPi)) : e;
}
template <typename T> __device__ __forceinline__ T wrap_angle(T a) {  // simple_env.py:63-65
  T s, c;
  m_sincos(a, &s, &c);
  return m_atan2(s, c);
}
// f32 build: atan2(sin a, cos a) == a - 2 pi rint(a / 2 pi) up to rounding (|err| ~ ulp(a))
template <> __device__ __forceinline__ float wrap_angle(float a) {
  return fmaf(-6.28318548f, rintf(a * 0.159154943f), a);
}

// ----------------------------------------------------------------------------- wave helpers
__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ float bcast(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
__device__ __forceinline__ double bcast(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }
// wave64 ballot of a bool straight from its lane mask (HIP's __ballot(int) round-trips the
// predicate through a VGPR: v_cndmask + v_cmp_ne per call)
__device__ __forceinline__ unsigned long long ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

template <typename R> struct Bits;
template <> struct Bits<float> { using T = unsigned int; };
template <> struct Bits<double> { using T = unsigned long long; };
// ds_permute (push): this lane's value goes to lane `dst`; lanes nobody writes read 0.
__device__ __forceinline__ unsigned int permute(int dst, unsigned int v) {
  return (unsigned int)__builtin_amdgcn_ds_permute(dst << 2, (int)v);
}
__device__ __forceinline__ unsigned long long permute(int dst, unsigned long long v) {
  const unsigned int lo = permute(dst, (unsigned int)v), hi = permute(dst, (unsigned int)(v >> 32));
  return ((unsigned long long)hi << 32) | lo;
}

// DPP lane moves (gfx9 dpp_ctrl encodings): quad_perm [1,0,3,2], [2,3,0,1],
// row_half_mirror, row_mirror.  Inactive/out-of-row sources keep `v` (bound_ctrl off).
template <int CTRL> __device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL> __device__ __forceinline__ double dpp(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp((int)(b & 0xffffffffll), (int)(b & 0xffffffffll), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(b >> 32), (int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppHalfMirror = 0x141, kDppMirror = 0x140;

template <typename T> __device__ __forceinline__ T tmin(T a, T b) { return b < a ? b : a; }
template <typename T> __device__ __forceinline__ T tmax(T a, T b) { return b > a ? b : a; }

// Wave-wide min / max, result wave-uniform: 4 DPP steps reduce each 16-lane row, then the
// four row results are combined through v_readlane (no LDS round trips).
template <typename T> __device__ __forceinline__ T wave_min(T v) {
  v = tmin(v, dpp<kDppXor1>(v));
  v = tmin(v, dpp<kDppXor2>(v));
  v = tmin(v, dpp<kDppHalfMirror>(v));
  v = tmin(v, dpp<kDppMirror>(v));
  return tmin(tmin(bcast(v, 0), bcast(v, 16)), tmin(bcast(v, 32), bcast(v, 48)));
}
template <typename T> __device__ __forceinline__ T wave_max(T v) {
  v = tmax(v, dpp<kDppXor1>(v));
  v = tmax(v, dpp<kDppXor2>(v));
  v = tmax(v, dpp<kDppHalfMirror>(v));
  v = tmax(v, dpp<kDppMirror>(v));
  return tmax(tmax(bcast(v, 0), bcast(v, 16)), tmax(bcast(v, 32), bcast(v, 48)));
}

// ----------------------------------------------------------------------------- Philox RNG
// Counter-based Philox4x32-10: key = run seed, counter = (global env id, episode, draw).
// Resets are reproducible per (seed, global env id, episode) and independent of how the
// envs are sharded over GPUs.  The reference draws from numpy PCG64 (simple_env.py:228-308);
// parity of resets is distributional (tests/test_gpu_parity.py KS tests).
struct Philox {
  uint32_t c0, c1, c2, c3, k0, k1;
  double spare;
  bool has_spare;

  __device__ Philox(uint64_t seed, uint64_t gid, uint32_t episode)
      : c0((uint32_t)gid), c1((uint32_t)(gid >> 32)), c2(episode), c3(0),
        k0((uint32_t)seed), k1((uint32_t)(seed >> 32)), spare(0.0), has_spare(false) {}

  __device__ void block(uint32_t& o0, uint32_t& o1, uint32_t& o2, uint32_t& o3) {
    uint32_t x0 = c0, x1 = c1, x2 = c2, x3 = c3, a = k0, b = k1;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      const uint32_t lo0 = 0xD2511F53u * x0, hi0 = __umulhi(0xD2511F53u, x0);
      const uint32_t lo1 = 0xCD9E8D57u * x2, hi1 = __umulhi(0xCD9E8D57u, x2);
      x0 = hi1 ^ x1 ^ a; x1 = lo1; x2 = hi0 ^ x3 ^ b; x3 = lo0;
      a += 0x9E3779B9u; b += 0xBB67AE85u;
    }
    ++c3;
    o0 = x0; o1 = x1; o2 = x2; o3 = x3;
  }
  // uniform double in [0, 1) with 53 random bits
  __device__ double uniform() {
    if (has_spare) { has_spare = false; return spare; }
    uint32_t a, b, c, d;
    block(a, b, c, d);
    const double s = 1.0 / 9007199254740992.0;  // 2^-53
    spare = (double)((((uint64_t)c << 32) | d) >> 11) * s;
    has_spare = true;
    return (double)((((uint64_t)a << 32) | b) >> 11) * s;
  }
  __device__ double uniform(double lo, double hi) { return lo + (hi - lo) * uniform(); }
  __device__ double normal(double mean, double scale) {  // Box-Muller
    const double u1 = 1.0 - uniform(), u2 = uniform();
    return mean + scale * sqrt(-2.0 * log(u1)) * cos(2.0 * kPi * u2);
  }
  __device__ int integers(int lo, int hi) {  // [lo, hi)
    int v = lo + (int)(uniform() * (double)(hi - lo));
    return v < hi ? v : hi - 1;
  }
};

// ----------------------------------------------------------------------------- ASMC
// One UsvAsmc.compute substep (usv_asmc.py:56-242, do_perturb = False).  State `s` holds
// the 16 unique values: psi_d_last, o, o', o'', eta_dot_last[3], upsilon_dot_last[3],
// e_u_last, Ka_dot_u_last, Ka_dot_psi_last, e_u_int, Ka_u, Ka_psi.
// do_perturb force of substep `pstep` (usv_asmc.py:184-199): t = perturb_step * integral_step,
// k = freq * 2 pi, F = (cos(t k), cos(t + k + 10)) * magnitude (the `t + k + 10` is the
// reference's), rotated as the row vector F @ J(psi).  Evaluated in double in both builds (t k
// reaches ~1e4 rad within an episode).
__device__ __forceinline__ void perturb_force(int pstep, double& fx, double& fy) {
  const double t = (double)pstep * H;
  const double k = 10.0 * (2.0 * kPi);
  fx = cos(t * k) * 5.0;
  fy = cos(t + k + 10.0) * 5.0;
}

// Trapezoid update H (a + b) / 2 + c (usv_asmc.py:87-88, 129, 143-146, 228-234).  f32 build: one
// fused multiply-add by H / 2 (the product H (a + b) / 2 equals (a + b) * fl(H / 2) before the final
// rounding); f64 build: the reference's operation order, bit-exact vs the oracle.
__device__ __forceinline__ float  asmc_trap(float a, float b, float c)  { return fmaf(a + b, 0.005f, c); }
__device__ __forceinline__ double asmc_trap(double a, double b, double c) { return H * (a + b) / 2.0 + c; }
// k * np.sign(d) for the adaptive gains (usv_asmc.py:137-140); f32: copysign (np.sign(0) = 0 kept)
__device__ __forceinline__ float  asmc_ksign(float k, float d)  { return d != 0.0f ? copysignf(k, d) : 0.0f; }
__device__ __forceinline__ double asmc_ksign(double k, double d) { return k * m_sign(d); }
// -K sqrt|sig| sign(sig) (usv_asmc.py:150-151); f32: copysign of the root (equal but for the sign of
// a zero result, which the following subtraction absorbs)
__device__ __forceinline__ float  asmc_root(float K, float sig)  { return -K * copysignf(__builtin_amdgcn_sqrtf(fabsf(sig)), sig); }
__device__ __forceinline__ double asmc_root(double K, double sig) { return -K * sqrt(fabs(sig)) * m_sign(sig); }
// wrap_once (usv_asmc.py:120); f32: e - copysign(2 pi, e), bit-identical to sign(e) (|e| - 2 pi)
__device__ __forceinline__ float  asmc_wrap(float e)  { return fabsf(e) > float(kPi) ? e - copysignf(float(2 * kPi), e) : e; }
__device__ __forceinline__ double asmc_wrap(double e) { return wrap_once(e); }

template <typename R>
__device__ __forceinline__ void asmc_substep(R (&s)[kAsmcN], R a0, R a1, R& x, R& y, R& psi,
                                             R& u, R& v, R& r, int pstep = 0, bool perturb = false) {
  // f32 build: hardware sqrt / reciprocal / sin / cos and constant reciprocals (the f64 build
  // keeps IEEE division and libm, bit-exact vs the oracle); hypot == sqrt(u^2 + v^2) here
  const R vmag = fx_sqrt(u * u + v * v);
  const R speed = std::is_same<R, float>::value ? vmag : m_hypot(u, v);
  const R beta = m_asin(fx_div(v, R(0.001) + speed));                     // :72
  const R psi_d = psi + beta + a1;                                         // :73-77
  R r_d = fx_cdiv(psi_d - s[0], H);                                        // :84
  s[0] = psi_d;
  const R o_dd = ((r_d - s[1]) * R(F1) - R(F3) * s[2]) * R(F2);            // :86
  const R o_d = asmc_trap(o_dd, s[3], s[2]);                        // :87
  const R o = asmc_trap(o_d, s[2], s[1]);                           // :88
  s[1] = o; s[2] = o_d; s[3] = o_dd;
  r_d = o;                                                                 // :89
  const bool fast = m_abs(u) > R(1.2);                                     // :95-99
  const R xu = fast ? R(64.55) : R(-25.0);
  const R xuu = fast ? R(-70.92) : R(0.0);
  const R yv = R(YV_K) * m_abs(v);                                         // :101-102
  const R yr = R(YR_K) * vmag, nv = R(NV_K) * vmag, nr = R(NR_K) * vmag;  // :103-108
  const R f_u = fx_cdiv(R(MASS - Y_V_DOT) * v * r + (xuu * m_abs(u) + xu * u), MASS - X_U_DOT);  // :113
  const R f_psi = fx_cdiv(R(-X_U_DOT + Y_V_DOT) * u * v + nr * r, IZ - N_R_DOT);                 // :115
  const R e_psi = asmc_wrap(psi_d - psi);                                  // :119-120
  const R e_psi_dot = r_d - r;                                             // :121
  const R e_u = a0 - u;                                                    // :128
  s[13] = asmc_trap(e_u, s[10], s[13]);                             // :129 e_u_int
  s[10] = e_u;
  const R sig_u = e_u + R(LAMBDA_U) * s[13];                               // :133
  const R sig_p = e_psi_dot + R(LAMBDA_PSI) * e_psi;                       // :134
  const R kdu = s[14] > R(KMIN_U) ? asmc_ksign(R(K_U), m_abs(sig_u) - R(MU_U)) : R(KMIN_U);       // :137
  const R kdp = s[15] > R(KMIN_PSI) ? asmc_ksign(R(K_PSI), m_abs(sig_p) - R(MU_PSI)) : R(KMIN_PSI);
  s[14] = asmc_trap(kdu, s[11], s[14]);                             // :143
  s[15] = asmc_trap(kdp, s[12], s[15]);                             // :146
  s[11] = kdu; s[12] = kdp;
  const R ua_u = asmc_root(s[14], sig_u) - R(K2_U) * sig_u;   // :150
  const R ua_p = asmc_root(s[15], sig_p) - R(K2_PSI) * sig_p; // :151
  const R tx = (R(LAMBDA_U) * e_u - f_u - ua_u) * R(MASS - X_U_DOT);      // :154
  const R tz = (R(LAMBDA_PSI) * e_psi - f_psi - ua_p) * R(IZ - N_R_DOT);  // :155
  const R tport = tx / R(2) + fx_cdiv(tz, B_TH);                           // :158
  const R tstbd = fx_cdiv(tx, 2 * C_TH) - fx_cdiv(tz, B_TH * C_TH);        // :159
  const R t0 = tport + R(C_TH) * tstbd;                                    // :176
  const R t2 = R(0.5 * B_TH) * (tport - R(C_TH) * tstbd);
  // rhs = T - C(nu) nu - D(nu) nu with C = CRB + CA (:201-211), D = Dl - Dn (:213-223)
  const R c02 = R(-MASS) * v + R(2) * (R(Y_V_DOT) * v + R((Y_R_DOT + N_V_DOT) / 2) * r);
  const R c12 = R(MASS) * u - R(X_U_DOT * MASS) * u;
  const R c20 = R(MASS) * v + R(2) * (R(-Y_V_DOT) * v - R((Y_R_DOT + N_V_DOT) / 2) * r);
  const R c21 = R(-MASS) * u + R(X_U_DOT * MASS) * u;
  const R av = m_abs(v), ar = m_abs(r);
  const R d00 = -xu - xuu * m_abs(u);
  const R d11 = -yv - (R(YVV) * av + R(YVR) * ar);
  const R d12 = -yr - (R(YRV) * av + R(YRR) * ar);
  const R d21 = -nv - (R(NVV) * av + R(NVR) * ar);
  const R d22 = -nr - (R(NRV) * av + R(NRR) * ar);
  R sp, cp;
  fx_sincos(psi, &sp, &cp);                                                // J(psi_old) :179
  R tt0 = t0, tt1 = R(0);
  if (perturb) {                                                           // T += F @ J (:184-198)
    double fx, fy;
    perturb_force(pstep, fx, fy);
    const R pfx = R(fx), pfy = R(fy);
    tt0 = t0 + (pfx * cp + pfy * sp);
    tt1 = R(0) + (pfx * -sp + pfy * cp);
  }
  const R rhs0 = tt0 - c02 * r - d00 * u;
  const R rhs1 = tt1 - c12 * r - (d11 * v + d12 * r);
  const R rhs2 = t2 - (c20 * u + c21 * v) - (d21 * v + d22 * r);
  const R ud = R(MI00) * rhs0;                                             // :226
  const R vd = R(MI11) * rhs1 + R(MI12) * rhs2;
  const R rd = R(MI21) * rhs1 + R(MI22) * rhs2;
  u = asmc_trap(ud, s[7], u);                                       // :228-229
  v = asmc_trap(vd, s[8], v);
  r = asmc_trap(rd, s[9], r);
  s[7] = ud; s[8] = vd; s[9] = rd;
  const R xd = cp * u - sp * v, yd = sp * u + cp * v, pd = r;              // :233
  x = asmc_trap(xd, s[4], x);                                       // :234
  y = asmc_trap(yd, s[5], y);
  psi = asmc_trap(pd, s[6], psi);
  s[4] = xd; s[5] = yd; s[6] = pd;
}


// f32 build of asmc_substep: the same law with its algebra folded.  Each rewrite is an identity in
// real arithmetic, so the float result differs from the reference-order evaluation by rounding
// only (the f64 build keeps asmc_substep above, bit-exact vs the oracle):
//  * the thruster split and its recombination (usv_asmc.py:158-159, 176) is the identity
//    T = (Tx, 0, Tz);
//  * Tx = (m - Xu')(lambda_u e_u - f_u - ua_u) with f_u = [...] / (m - Xu') (:113, :154): the
//    division and the multiplication cancel (likewise Iz - Nr' in Tz, :115, :155);
//  * C(nu) (:201-211): c20 = -c02 and c21 = -c12; D(nu) (:213-223): each entry one linear form in
//    |v|, |r| and |nu| with the scale factors of :101-108 folded into its coefficients;
//  * trapezoids H (a + b) / 2 + c as one fma by H / 2; ((r_d - o) F1 - F3 o') F2 with F = 2 as
//    4 ((r_d - o) - o') (:86; bit-identical); np.sign products as copysign.
//  * a ~50 m float position rounded at each of the 20 substeps was the f32 path's largest error (the
//    reward's ye term amplifies it), so the pose is rounded once per run of substeps: x and y are not
//    read inside the substep, so they accumulate in xl, yl and the caller applies them after the run;
//    psi is read by the next substep, so it also integrates as usual and pl carries the correction
//    (round 3, v1: the increments, with psi's compensated summation; golden replay reward error
//    1.0e-4 -> 3.5e-5; round 5, v2: the rates, telescoped below).
// End of a run of f32 substeps: the pose from what asmc_substep_f32 accumulated.  Round 5: xl, yl, pl
// are the sums of the rates x', y', r over the run, and each trapezoid sum is telescoped,
// sum_k h2 (q_k + q_{k-1}) = h2 (2 sum - q_last + q_{-1}) (q_{-1} = s[4], s[5], s[6] before the run:
// e0 = {x4, y5, r6}); psi0 is the heading before the run (inside the run psi integrates as usual,
// since the substeps read it).  v1: xl, yl the increments, pl the compensated summation's error.
struct AsmcRun { float x4, y5, r6, psi0; };
__device__ __forceinline__ AsmcRun asmc_run_begin(const float (&s)[kAsmcN], float psi) {
  return AsmcRun{s[4], s[5], s[6], psi};
}
__device__ __forceinline__ void asmc_run_end(float& x, float& y, float& psi, float xl, float yl, float pl,
                                             const AsmcRun& e0, const float (&s)[kAsmcN]) {
  constexpr float h2 = float(H / 2);
  x += h2 * (fmaf(2.0f, xl, -s[4]) + e0.x4);
  y += h2 * (fmaf(2.0f, yl, -s[5]) + e0.y5);
  psi = e0.psi0 + h2 * (fmaf(2.0f, pl, -s[6]) + e0.r6);
}

// asin on [-1, 1] for the f32 substep: |x| < 1/2 as s + s t P(t) with t = x^2, else
// pi/2 - 2 asin(sqrt((1 - |x|) / 2)) with the same polynomial (Cephes asinf's minimax P, ~2.5e-7
// relative); one hardware sqrt, both arms branch-free
__device__ __forceinline__ float asin_f32(float x) {
  const float ax = fabsf(x);
  const bool big = ax >= 0.5f;
  const float t = big ? fmaf(-0.5f, ax, 0.5f) : x * x;
  const float s = big ? __builtin_amdgcn_sqrtf(t) : ax;
  const float p = fmaf(fmaf(fmaf(fmaf(4.2163199048e-2f, t, 2.4181311049e-2f), t, 4.5470025998e-2f), t,
                            7.4953002686e-2f), t, 1.6666752422e-1f);
  const float as = fmaf(s * t, p, s);
  return copysignf(big ? fmaf(-2.0f, as, 1.57079632679f) : as, x);
}

// Round 5: the rhs of M nu' = tau - C(nu) nu - D(nu) nu folded further (identities in real arithmetic,
// with (Tx, 0, Tz) as in round 4):
//  * surge: M00 = m - Xu', so u' = (lambda_u e_u - ua_u) - (Yv' v r + (Yr' + Nv') r^2 + Xuu |u| (1 - u)) / M00
//    (f_u's and C's v r terms and D's Xu u cancel: the reference's f_u carries Xuu |u| + Xu u, :113);
//  * yaw: tau_z's -Nr r cancels D's Nr-linear part (:108, :213-223), and the u v terms of tau_z and
//    C(nu) are one coefficient;
//  * np.sign(|sigma| - mu) at exactly 0 is not kept (the f32 equality is not the reference's float64
//    one anyway);  asin as asin_f32 above.
// The f32 substep is held to SURVEY 8(c)'s tolerance, not to the reference's rounding.
__device__ __forceinline__ void asmc_substep_f32(float (&s)[kAsmcN], float a0, float a1, float& x, float& y,
                                                 float& psi, float& u, float& v, float& r, float& xl, float& yl,
                                                 float& pl, float kt, int pstep = 0, bool perturb = false) {
  constexpr float h2 = float(H / 2);
  const float au = fabsf(u), av = fabsf(v), ar = fabsf(r);
  const float vmag = __builtin_amdgcn_sqrtf(fmaf(u, u, v * v));
  // yaw channel: LOS heading, third-order filter, sliding surface (:72-89, :119-121, :134)
  const float beta = asin_f32(v * __builtin_amdgcn_rcpf(0.001f + vmag));
  const float ba = beta + a1;                                                   // psi_d - psi (:119)
  const float psi_d = psi + ba;
  const float r_d = (psi_d - s[0]) * float(1.0 / H);
  s[0] = psi_d;
  const float o_dd = 4.0f * ((r_d - s[1]) - s[2]);
  const float o_d = fmaf(o_dd + s[3], h2, s[2]);
  const float o = fmaf(o_d + s[2], h2, s[1]);
  s[1] = o; s[2] = o_d; s[3] = o_dd;
  const float e_psi = asmc_wrap(ba);
  const float sig_p = (o - r) + float(LAMBDA_PSI) * e_psi;
  // surge channel (:128-133)
  const float e_u = a0 - u;
  s[13] = fmaf(e_u + s[10], h2, s[13]);
  s[10] = e_u;
  const float sig_u = fmaf(float(LAMBDA_U), s[13], e_u);
  // adaptive gains (:137-146) and control laws (:150-151)
  const float kdu = s[14] > float(KMIN_U) ? copysignf(float(K_U), fabsf(sig_u) - float(MU_U)) : float(KMIN_U);
  const float kdp = s[15] > float(KMIN_PSI) ? copysignf(float(K_PSI), fabsf(sig_p) - float(MU_PSI)) : float(KMIN_PSI);
  s[14] = fmaf(kdu + s[11], h2, s[14]);
  s[15] = fmaf(kdp + s[12], h2, s[15]);
  s[11] = kdu; s[12] = kdp;
  const float au_u = fmaf(float(K2_U), sig_u, fmaf(float(LAMBDA_U), e_u,
                          s[14] * copysignf(__builtin_amdgcn_sqrtf(fabsf(sig_u)), sig_u)));   // lambda e - ua
  const float au_p = fmaf(float(K2_PSI), sig_p, fmaf(float(LAMBDA_PSI), e_psi,
                          s[15] * copysignf(__builtin_amdgcn_sqrtf(fabsf(sig_p)), sig_p)));
  // J(psi_old) (:179): v_sin / v_cos take revolutions; psi / 2 pi less the env step's whole turns kt
  // (the round-4 note above) in one fma: its error, |psi| 3e-8 / 2 pi revolutions, stays below half
  // an ulp of psi itself
  const float rev = fmaf(psi, float(1.0 / (2 * kPi)), -kt);
  const float sp = __builtin_amdgcn_sinf(rev), cp = __builtin_amdgcn_cosf(rev);
  float p0 = 0.0f, p1 = 0.0f;
  if (perturb) {                                                                // T += F @ J (:184-198)
    double fx, fy;
    perturb_force(pstep, fx, fy);
    const float pfx = float(fx), pfy = float(fy);
    p0 = pfx * cp + pfy * sp;
    p1 = pfx * -sp + pfy * cp;
  }
  const float xuu = au > 1.2f ? -70.92f : 0.0f;                                 // :95-99 (Xu cancels)
  const float qs = fmaf(xuu * au, 1.0f - u, fmaf(float(Y_R_DOT + N_V_DOT), r, float(Y_V_DOT) * v) * r);
  const float ud = perturb ? fmaf(float(MI00), p0 - qs, au_u) : fmaf(float(-MI00), qs, au_u);  // :226
  const float md11 = fmaf(float(YV_K + YVV), av, float(YVR) * ar);
  const float md12 = fmaf(float(YR_K), vmag, fmaf(float(YRV), av, float(YRR) * ar));
  const float md21 = fmaf(float(NV_K), vmag, fmaf(float(NVV), av, float(NVR) * ar));
  const float n22 = fmaf(float(NRV), av, float(NRR) * ar);
  const float rhs1 = fmaf(md11, v, fmaf(fmaf(float(-(MASS - X_U_DOT * MASS)), u, md12), r, p1));
  const float rhs2 = fmaf(float(IZ - N_R_DOT), au_p,
                          fmaf(u, fmaf(float(X_U_DOT + Y_V_DOT - X_U_DOT * MASS), v, float(Y_R_DOT + N_V_DOT) * r),
                               fmaf(md21, v, n22 * r)));
  const float vd = fmaf(float(MI11), rhs1, float(MI12) * rhs2);
  const float rd = fmaf(float(MI21), rhs1, float(MI22) * rhs2);
  u = fmaf(ud + s[7], h2, u);                                                   // :228-229
  v = fmaf(vd + s[8], h2, v);
  r = fmaf(rd + s[9], h2, r);
  s[7] = ud; s[8] = vd; s[9] = rd;
  const float xd = fmaf(cp, u, -(sp * v)), yd = fmaf(sp, u, cp * v);          // :233
  {                                                                             // :234
    // xl, yl, pl sum the rates; the caller applies the telescoped trapezoid sums once (asmc_run_end)
    xl += xd;
    yl += yd;
    pl += r;
    psi = fmaf(r + s[6], h2, psi);
  }
  s[4] = xd; s[5] = yd; s[6] = r;
}

}  // namespace usv
