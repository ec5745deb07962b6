// Same-address atomic throughput as the vertex kernels use it: every wave of a
// large grid appends (ballot, one atomicAdd by the leader) K times to one
// counter, or to one of S counters.  Prints the kernel time per config.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_append(int* ctr, int* out, int k_iters, int spread) {
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  int acc = 0;
  for (int k = 0; k < k_iters; ++k) {
    const bool want = ((lane * 7 + k * 13 + wave) % 3) != 0;
    const unsigned long long m = __ballot(want);
    if (m == 0ull) continue;
    const int leader = __ffsll(m) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(ctr + 64 * ((wave + k) % spread), __popcll(m));
    base = __shfl(base, leader);
    acc += base;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  const int waves = 40960, block = 256, grid = waves * 64 / block;
  int *ctr, *out;
  hipMalloc(&ctr, 64 * 64 * sizeof(int));
  hipMalloc(&out, size_t(grid) * block * sizeof(int));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int spread : {1, 8, 64}) {
    for (int k : {0, 1, 4, 8, 16}) {
      float best = 1e9f;
      for (int rep = 0; rep < 5; ++rep) {
        hipMemset(ctr, 0, 64 * 64 * sizeof(int));
        hipEventRecord(a);
        hipLaunchKernelGGL(k_append, dim3(grid), dim3(block), 0, 0, ctr, out, k, spread);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0.f;
        hipEventElapsedTime(&ms, a, b);
        best = ms < best ? ms : best;
      }
      std::printf("waves %d appends/wave %2d counters %2d: %8.1f us  (%.2f ns per atomic)\n", waves, k, spread,
                  best * 1e3f, k ? best * 1e6f / (double(waves) * k) : 0.0);
    }
  }
  return 0;
}
