// Microbenchmark (diagnostic, not the product): does reading only the first `pieces` 16-B pieces of
// each 384-B row fetch fewer bytes from memory than reading whole rows?  One wave per row-pair group,
// lane c reads piece c of a row (global_load_dwordx4), sums into one float per row (kept live).
//   hipcc -O3 --offload-arch=gfx950 tools/micro/fetch_granularity.hip -o diagbuild/fetch_gran
//   rocprofv3 --pmc FETCH_SIZE -- diagbuild/fetch_gran 24    (then 17, 9)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void rows_kernel(const float4* __restrict__ rows, float* __restrict__ out, int nrows, int pieces) {
  const int row = blockIdx.x * 4 + threadIdx.x / 64;
  const int c = threadIdx.x & 63;
  if (row >= nrows) return;
  float acc = 0.f;
  if (c < pieces) {
    const float4 v = rows[(size_t)row * 24 + c];
    acc = v.x + v.y + v.z + v.w;
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (c == 0) out[row] = acc;
}

int main(int argc, char** argv) {
  const int pieces = argc > 1 ? atoi(argv[1]) : 24;
  const int nrows = 524288;
  float4* rows;
  float* out;
  if (hipMalloc(&rows, (size_t)nrows * 384) != hipSuccess || hipMalloc(&out, nrows * 4) != hipSuccess) return 1;
  hipMemset(rows, 0, (size_t)nrows * 384);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int it = 0; it < 20; ++it) {
    // evict the Infinity Cache between passes with a 512 MB sweep every other launch
    hipLaunchKernelGGL(rows_kernel, dim3(nrows / 4), dim3(256), 0, 0, rows, out, nrows, pieces);
  }
  hipEventRecord(a);
  for (int it = 0; it < 20; ++it)
    hipLaunchKernelGGL(rows_kernel, dim3(nrows / 4), dim3(256), 0, 0, rows, out, nrows, pieces);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  printf("pieces %d: %.2f us per launch, useful %.1f MB per launch\n", pieces, ms * 1000 / 20,
         (double)nrows * pieces * 16 / 1e6);
  hipFree(rows);
  hipFree(out);
  return 0;
}
