// Workgroups resident per CU as a function of dynamic LDS bytes (256-thread
// workgroups): hipOccupancyMaxActiveBlocksPerMultiprocessor next to the peak
// residency measured from s_memrealtime begin/end stamps + HW_ID of a
// spinning kernel. Build: hipcc --offload-arch=gfx950 -O3 -o lds_occ lds_occupancy.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <map>
#include <vector>

__global__ __launch_bounds__(256) void k_spin(unsigned long long* st, unsigned* id, int spin) {
  extern __shared__ uint8_t lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  lds[threadIdx.x] = (uint8_t)threadIdx.x;
  __syncthreads();
  while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin) __builtin_amdgcn_s_sleep(4);
  if (threadIdx.x == 0) {
    unsigned xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    st[2 * blockIdx.x] = t0;
    st[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    id[blockIdx.x] = ((xcc & 15) << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15);
  }
  if (lds[(threadIdx.x + 1) & 255] == 0xff) st[0] = 0;
}

int main() {
  const int nwg = 4096;
  unsigned long long* st;
  unsigned* id;
  hipMalloc(&st, 2 * nwg * sizeof(unsigned long long));
  hipMalloc(&id, nwg * sizeof(unsigned));
  hipFuncSetAttribute((const void*)k_spin, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  std::vector<unsigned long long> hs(2 * nwg);
  std::vector<unsigned> hid(nwg);
  for (int bytes : {8192, 10240, 12288, 16384, 17408, 18200, 18432, 19456, 19656, 20000, 20224, 20480, 20481, 21504, 23040, 32768}) {
    int occ = -1;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_spin, 256, bytes);
    hipLaunchKernelGGL(k_spin, dim3(nwg), dim3(256), bytes, 0, st, id, 2000);  // 20 us
    hipDeviceSynchronize();
    hipMemcpy(hs.data(), st, hs.size() * 8, hipMemcpyDeviceToHost);
    hipMemcpy(hid.data(), id, hid.size() * 4, hipMemcpyDeviceToHost);
    std::map<unsigned, std::vector<std::pair<unsigned long long, int>>> ev;
    for (int w = 0; w < nwg; ++w) {
      ev[hid[w]].push_back({hs[2 * w], 1});
      ev[hid[w]].push_back({hs[2 * w + 1], -1});
    }
    int pmin = 1 << 30, pmax = 0;
    for (auto& kv : ev) {
      auto& v = kv.second;
      std::sort(v.begin(), v.end(), [](auto a, auto b) { return a.first != b.first ? a.first < b.first : a.second < b.second; });
      int live = 0, best = 0;
      for (auto& e : v) best = std::max(best, live += e.second);
      pmin = std::min(pmin, best);
      pmax = std::max(pmax, best);
    }
    printf("lds %6d B: occupancy API %d, measured peak resident per CU %d..%d over %zu CUs\n", bytes, occ, pmin, pmax,
           ev.size());
  }
  return 0;
}
