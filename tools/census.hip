// census.hip - how many one-wave workgroups of a given LDS / VGPR / SGPR
// footprint the MI355X keeps resident at once (diagnostic, tools/ only).
//
//   hipcc --offload-arch=gfx950 -O2 tools/census.hip -o build/census && build/census
//
// Each workgroup bumps a global "alive" counter, records the running maximum,
// holds its slot for ~300 us of s_sleep, then leaves.  The grid is larger
// than any plausible residency, so the maximum is the residency.
#include <hip/hip_runtime.h>

#include <cstdio>

template <int kLds, int kV>
__global__ __launch_bounds__(64) void k_census(unsigned* alive, unsigned* peak, unsigned long long t_end) {
  __shared__ unsigned pad[kLds / 4];
  if (kV == 96) asm volatile("" ::: "v95");
  if (kV == 104) asm volatile("" ::: "v103");
  if (kV == 128) asm volatile("" ::: "v127");
  asm volatile("" ::: "s101");
  pad[threadIdx.x] = threadIdx.x;
  if (threadIdx.x == 0) {
    const unsigned a = atomicAdd(alive, 1u) + 1u;
    atomicMax(peak, a);
  }
  while (__builtin_amdgcn_s_memrealtime() < t_end) __builtin_amdgcn_s_sleep(20);
  if (threadIdx.x == 0) atomicSub(alive, 1u);
  if (pad[(threadIdx.x + 1) & 63] == 12345u) alive[1] = 0;
}

__global__ void k_now(unsigned long long* p) { *p = __builtin_amdgcn_s_memrealtime(); }

template <int kLds, int kV>
void run(const char* name) {
  unsigned *d, h[2];
  hipMalloc(&d, 16);
  hipMemset(d, 0, 16);
  // end time: now + 3 ms in the 100 MHz realtime counter, read on the device
  unsigned long long* dt;
  hipMalloc(&dt, 8);
  hipLaunchKernelGGL(k_now, dim3(1), dim3(1), 0, 0, dt);
  unsigned long long now;
  hipMemcpy(&now, dt, 8, hipMemcpyDeviceToHost);
  hipLaunchKernelGGL((k_census<kLds, kV>), dim3(8192), dim3(64), 0, 0, d, d + 1, now + 300000ull);
  hipDeviceSynchronize();
  hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
  int occ = 0;
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_census<kLds, kV>, 64, 0);
  printf("%-22s LDS %6d B  VGPR %3d: peak resident %5u (%.2f per CU), occupancy API %d per CU\n", name, kLds, kV, h[1],
         h[1] / 256.0, occ);
  hipFree(d);
  hipFree(dt);
}

int main() {
  run<8192, 96>("5 waves, 8 KB");
  run<8064, 96>("5 waves, 8064 B");
  run<7936, 96>("5 waves, 7936 B");
  run<7680, 96>("5 waves, 7.5 KB");
  run<10240, 96>("4 waves, 10 KB");
  run<10112, 96>("4 waves, 10112 B");
  run<9984, 96>("4 waves, 9984 B");
  run<9728, 96>("4 waves, 9.5 KB");
  run<1024, 96>("VGPR 96 only");
  run<1024, 104>("VGPR 104 only");
  return 0;
}
