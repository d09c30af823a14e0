// coop_exit.hip -- the exit-time crash probe without torch: one hipLaunchCooperativeKernel
// with /opt/rocm's HIP runtime, then exit. Under rocprofv3 --kernel-trace this exits
// cleanly or not; tools/archive/exit_probe.sh compares it with the torch-hosted probe.
//   hipcc --offload-arch=gfx950 -O2 -o build/coop_exit tools/archive/coop_exit.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(int *x) { atomicAdd(x, 1); }

int main() {
  int *d;
  if (hipMalloc(&d, 4) != hipSuccess) return 1;
  hipMemset(d, 0, 4);
  void *args[] = {&d};
  hipError_t e = hipLaunchCooperativeKernel((const void *)k, dim3(64), dim3(64), args, 0, 0);
  int h = 0;
  hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
  printf("cooperative launch: %s, %d lanes\n", hipGetErrorString(e), h);
  hipFree(d);
  return 0;
}
