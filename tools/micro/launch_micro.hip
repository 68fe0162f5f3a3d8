// Launch-overhead microbenchmark: empty / near-empty 256-thread workgroups with
// and without a large dynamic LDS allocation (how much of a short per-env
// kernel is dispatch and LDS-limited residency).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void k_empty(int* out) {
  if (threadIdx.x == 1023) out[blockIdx.x] = 1;
}
__global__ __launch_bounds__(256) void k_lds(int* out) {
  extern __shared__ int lds[];
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (lds[(threadIdx.x + 1) & 255] == 12345) out[blockIdx.x] = 1;
}
// a dependent global load chain of depth D per workgroup (record-read latency)
__global__ __launch_bounds__(256) void k_chain(const int* __restrict__ in, int* out, int D) {
  extern __shared__ int lds[];
  int v = blockIdx.x * 997;
  for (int d = 0; d < D; ++d) v = in[(v & 0xFFFFF) * 16];
  lds[threadIdx.x] = v;
  __syncthreads();
  if (lds[(threadIdx.x + 1) & 255] == 12345) out[blockIdx.x] = 1;
}

static float time_ms(void (*launch)(hipStream_t), hipStream_t s, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 5; ++i) launch(s);
  hipEventRecord(a, s);
  for (int i = 0; i < iters; ++i) launch(s);
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / iters;
}

static int* g_out;
static int* g_in;
static int g_n = 4096;
static size_t g_lds = 0;
static int g_D = 0;
static void L_empty(hipStream_t s) { hipLaunchKernelGGL(k_empty, dim3(g_n), dim3(256), g_lds, s, g_out); }
static void L_lds(hipStream_t s) { hipLaunchKernelGGL(k_lds, dim3(g_n), dim3(256), g_lds, s, g_out); }
static void L_chain(hipStream_t s) { hipLaunchKernelGGL(k_chain, dim3(g_n), dim3(256), g_lds, s, g_in, g_out, g_D); }

int main() {
  hipMalloc(&g_out, 1 << 24);
  hipMalloc(&g_in, 64 << 20);
  hipMemset(g_in, 0, 64 << 20);
  hipFuncSetAttribute((const void*)k_empty, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipFuncSetAttribute((const void*)k_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipFuncSetAttribute((const void*)k_chain, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipStream_t s;
  hipStreamCreate(&s);
  size_t ldss[] = {1024, 20 * 1024, 38592, 76 * 1024};
  for (size_t l : ldss) {
    g_lds = l;
    printf("lds=%6zu  empty %.2f us  lds+barrier %.2f us", l, 1e3 * time_ms(L_empty, s, 50), 1e3 * time_ms(L_lds, s, 50));
    for (int D : {1, 2, 4}) {
      g_D = D;
      printf("  chain%d %.2f us", D, 1e3 * time_ms(L_chain, s, 50));
    }
    printf("\n");
  }
  return 0;
}
