// usv_diag.hpp -- instrumentation of the DIAGNOSTIC builds only (tools/build_diag.sh: -DUSV_DIAG
// plus one of USV_DIAG_STAMPS / USV_DIAG_PROF / USV_DIAG_QPROF).  The product library never
// includes this file: usv_kernels.hip defines the same names as no-ops when USV_DIAG is unset.
// Stamps go to __device__ arrays of their own that no kernel output reads.
#pragma once
#ifndef USV_DIAG
#error "usv_diag.hpp is for the diagnostic builds only (-DUSV_DIAG)"
#endif

// (included inside namespace usv by usv_kernels.hip)

// Diagnostic build only (-DUSV_DIAG_STAMPS): per-block s_memrealtime (100 MHz) stamps at the
// phase boundaries of the step kernel, read back with usv_diag_stamps().  Never in the product.
#ifdef USV_DIAG_STAMPS
constexpr int kStampSlots = 8;
__device__ unsigned long long g_stamps[32768 * kStampSlots];
#define USV_STAMP(i)                                                                      \
  do {                                                                                    \
    if (threadIdx.x == 0 && blockIdx.x < 32768)                                           \
      g_stamps[blockIdx.x * kStampSlots + (i)] = __builtin_amdgcn_s_memrealtime();        \
  } while (0)
// block slot, written by the first lane of whichever wave executes it (kind 0)
#define USV_STAMP_B(i)                                                                    \
  do {                                                                                    \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 32768)                                    \
      g_stamps[blockIdx.x * kStampSlots + (i)] = __builtin_amdgcn_s_memrealtime();        \
  } while (0)
// wave slot (global wave index; kinds 1-3)
#define USV_STAMP_W(i)                                                                    \
  do {                                                                                    \
    const unsigned gw_ = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;               \
    if ((threadIdx.x & 63) == 0 && gw_ < 32768)                                           \
      g_stamps[gw_ * kStampSlots + (i)] = __builtin_amdgcn_s_memrealtime();               \
  } while (0)
// a wave slot holding a value instead of a time
#define USV_STAMP_V(i, v)                                                                 \
  do {                                                                                    \
    const unsigned gw_ = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;               \
    if ((threadIdx.x & 63) == 0 && gw_ < 32768) g_stamps[gw_ * kStampSlots + (i)] = (v);  \
  } while (0)
// slot 7: HW_ID (SIMD, CU, SE bits) | XCC_ID << 32 of the wave
#define USV_STAMP_ID()                                                                    \
  do {                                                                                    \
    const unsigned gw_ = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;               \
    const unsigned long long hw_ = __builtin_amdgcn_s_getreg((31 << 11) | 4);             \
    const unsigned long long xcc_ = __builtin_amdgcn_s_getreg((15 << 11) | 20);           \
    if ((threadIdx.x & 63) == 0 && gw_ < 32768) g_stamps[gw_ * kStampSlots + 7] = hw_ | (xcc_ << 32); \
  } while (0)
#else
#define USV_STAMP_ID() do {} while (0)
#define USV_STAMP(i) do {} while (0)
#define USV_STAMP_B(i) do {} while (0)
#define USV_STAMP_W(i) do {} while (0)
#define USV_STAMP_V(i, v) do {} while (0)
#endif
// Diagnostic build only (-DUSV_DIAG_PROF): per-wave shader-clock (s_memtime) cycles spent in
// each part of the wave-per-env scan, read back with usv_diag_prof().  Never in the product.
#ifdef USV_DIAG_PROF
constexpr int kProfWaves = 16384, kProfSlots = 8;
__device__ unsigned long long g_prof[kProfWaves * kProfSlots];
struct Prof {
  unsigned long long acc[kProfSlots] = {};
  unsigned long long t;
  __device__ Prof() : t(__builtin_amdgcn_s_memtime()) {}
  __device__ void mark(int i) {
    const unsigned long long n = __builtin_amdgcn_s_memtime();
    acc[i] += n - t;
    t = n;
  }
  __device__ void count(int i) { acc[i] += 1; }
  __device__ void flush(int gw) {
    if ((threadIdx.x & 63) == 0 && gw < kProfWaves)
      for (int k = 0; k < kProfSlots; ++k) g_prof[gw * kProfSlots + k] = acc[k];
  }
};
#else
struct Prof {
  __device__ void mark(int) {}
  __device__ void count(int) {}
  __device__ void flush(int) {}
};
#endif
// Diagnostic build only (-DUSV_DIAG_QPROF): per-wave shader-clock cycles (s_memtime; its SMEM
// round trip also waits for the wave's LDS ops, so the marks perturb what they time) spent in each section of the block-queue step, read back with usv_diag_qprof().
#ifdef USV_DIAG_QPROF
constexpr int kQProfSlots = 12;
__device__ unsigned g_qprof[16384 * kQProfSlots];
__device__ __forceinline__ unsigned shader_cycles() { return (unsigned)__builtin_amdgcn_s_memtime(); }
struct QProf {
  unsigned acc[kQProfSlots];
  unsigned t;
  __device__ QProf() : t(shader_cycles()) { for (int i = 0; i < kQProfSlots; ++i) acc[i] = 0; }
  __device__ __forceinline__ void mark(int i) { const unsigned n = shader_cycles(); acc[i] += n - t; t = n; }
  __device__ __forceinline__ void count(int i, unsigned k = 1) { acc[i] += k; }
  __device__ void flush() {
    const unsigned gw = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    if ((threadIdx.x & 63) == 0 && gw < 16384)
      for (int k = 0; k < kQProfSlots; ++k) g_qprof[gw * kQProfSlots + k] = acc[k];
  }
};
#define QMARK(i) do { if (qp) qp->mark(i); } while (0)
__device__ __forceinline__ void qprof_flush(QProf* qp) { qp->flush(); }
#define QCOUNT(i, k) do { if (qp) qp->count(i, k); } while (0)
#else
struct QProf { __device__ void mark(int) {} __device__ void count(int, unsigned = 1) {} __device__ void flush() {} };
#ifdef USV_DIAG_SECTIONS
// (-DUSV_DIAG_SECTIONS, assembly listings only: a comment per section boundary for
// tools/section_mix.py's static instruction mix of the block-queue loop)
#define QMARK(i) asm volatile(";@@QMARK " #i)
#else
#define QMARK(i) do {} while (0)
#endif
#define QCOUNT(i, k) do {} while (0)
__device__ __forceinline__ void qprof_flush(QProf*) {}
#endif
