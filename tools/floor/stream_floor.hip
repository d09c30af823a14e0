// Diagnostic: the streaming floor of k_simulate's byte pattern (SP_Oracle shape, P = 2, E = 5):
// read ctx [5][B] f64, part [2][B] i32, u [B] f64 (56 B); write winner i32, price f64,
// outcome u8, item [2][B] i32, bid / est / true / best_ev [2][B] f64 (85 B) -- with trivial
// arithmetic, so the time is the memory system's. Two launch shapes: persistent grid-stride
// (as k_simulate) and one 256-auction tile per block.
#include <hip/hip_runtime.h>
#include <stdint.h>

struct Ptrs {
  const double *ctx;
  const int32_t *part;
  const double *u;
  int32_t *winner, *item;
  double *price, *bid, *est, *tru, *bev;
  uint8_t *outcome;
};

__device__ __forceinline__ void one(const Ptrs &p, int64_t B, int64_t i) {
  double x0 = p.ctx[i], x1 = p.ctx[B + i], x2 = p.ctx[2 * B + i], x3 = p.ctx[3 * B + i], x4 = p.ctx[4 * B + i];
  int a0 = p.part[i], a1 = p.part[B + i];
  double u = p.u[i];
  double s = x0 + x1 + x2 + x3 + x4;
  p.winner[i] = a0 > a1;
  p.price[i] = s * u;
  p.outcome[i] = (uint8_t)(u > 0.5);
  p.item[i] = a0;
  p.item[B + i] = a1;
  p.bid[i] = s;
  p.bid[B + i] = s + u;
  p.est[i] = x0;
  p.est[B + i] = x1;
  p.tru[i] = x2;
  p.tru[B + i] = x3;
  p.bev[i] = x4;
  p.bev[B + i] = u;
}

__global__ __launch_bounds__(256) void k_floor_persistent(Ptrs p, int64_t B) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < B; i += (int64_t)gridDim.x * 256) one(p, B, i);
}
__global__ __launch_bounds__(256) void k_floor_tiles(Ptrs p, int64_t B) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < B) one(p, B, i);
}

extern "C" int floor_run(int persistent, int grid, const Ptrs *p, int64_t B, void *stream) {
  if (persistent)
    hipLaunchKernelGGL(k_floor_persistent, dim3(grid), dim3(256), 0, (hipStream_t)stream, *p, B);
  else
    hipLaunchKernelGGL(k_floor_tiles, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream, *p, B);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
