// Do relaxed fetch_adds on one counter from waves on all XCDs return unique values?  agent scope
// (global_atomic_add sc0) against system scope (sc0 sc1); 512 blocks x 16 waves, lane 0 of each wave
// claims 8 times from counter blockIdx % 16.  Diagnostic for step_q_body's global pair claims.
//   hipcc --offload-arch=gfx950 -O2 -o xcd_atomics tools/micro/xcd_atomics.hip && ./xcd_atomics
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
template <int SCOPE>
__global__ void claims(unsigned* ctr, unsigned* out) {
  const int w = blockIdx.x * 16 + threadIdx.x / 64;
  if ((threadIdx.x & 63) != 0) return;
  unsigned* c = ctr + 32 * (blockIdx.x % 16);
  for (int i = 0; i < 8; ++i) out[w * 8 + i] = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, SCOPE);
}
int main() {
  const int nw = 512 * 16, n = nw * 8;
  unsigned *ctr, *out;
  if (hipMalloc(&ctr, 16 * 128) != hipSuccess || hipMalloc(&out, n * 4) != hipSuccess) return 2;
  std::vector<unsigned> h(n);
  for (int scope = 0; scope < 2; ++scope) {
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipMemset(ctr, 0, 16 * 128);
      if (scope == 0) hipLaunchKernelGGL(claims<__HIP_MEMORY_SCOPE_AGENT>, dim3(512), dim3(1024), 0, 0, ctr, out);
      else hipLaunchKernelGGL(claims<__HIP_MEMORY_SCOPE_SYSTEM>, dim3(512), dim3(1024), 0, 0, ctr, out);
      hipEvent_t a, b;
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(h.data(), out, n * 4, hipMemcpyDeviceToHost);
      int dup = 0, bad = 0;
      for (int k = 0; k < 16; ++k) {
        std::vector<unsigned> v;
        for (int w = 0; w < nw; ++w)
          if ((w / 16) % 16 == k)
            for (int i = 0; i < 8; ++i) v.push_back(h[w * 8 + i]);
        std::sort(v.begin(), v.end());
        for (size_t i = 0; i < v.size(); ++i) {
          if (i && v[i] == v[i - 1]) ++dup;
          if (v[i] >= v.size()) ++bad;
        }
      }
      printf("{\"scope\": \"%s\", \"rep\": %d, \"claims\": %d, \"duplicates\": %d, \"out_of_range\": %d}\n",
             scope ? "system" : "agent", rep, n, dup, bad);
      (void)a; (void)b;
    }
  }
  return 0;
}
