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

template <bool NT, typename T> __device__ __forceinline__ T L(const T *q) {
  if constexpr (NT) return __builtin_nontemporal_load(q); else return *q;
}
template <bool NT, typename T> __device__ __forceinline__ void S(T *q, T v) {
  if constexpr (NT) __builtin_nontemporal_store(v, q); else *q = v;
}
// WO: winner and outcome as one word (ABI 17 winner_outcome), no byte stream
template <bool NT = false, bool WO = false>
__device__ __forceinline__ void one(const Ptrs &p, int64_t B, int64_t i) {
  double x0 = L<NT>(p.ctx + i), x1 = L<NT>(p.ctx + B + i), x2 = L<NT>(p.ctx + 2 * B + i),
         x3 = L<NT>(p.ctx + 3 * B + i), x4 = L<NT>(p.ctx + 4 * B + i);
  int a0 = L<NT>(p.part + i), a1 = L<NT>(p.part + B + i);
  double u = L<NT>(p.u + i);
  double s = x0 + x1 + x2 + x3 + x4;
  if constexpr (WO) {
    S<NT>(p.winner + i, (int32_t)((uint32_t)(a0 > a1) | ((uint32_t)(u > 0.5) << 31)));
  } else {
    S<NT>(p.winner + i, (int32_t)(a0 > a1));
    S<NT>(p.outcome + i, (uint8_t)(u > 0.5));
  }
  S<NT>(p.price + i, s * u);
  S<NT>(p.item + i, (int32_t)a0);
  S<NT>(p.item + B + i, (int32_t)a1);
  S<NT>(p.bid + i, s);
  S<NT>(p.bid + B + i, s + u);
  S<NT>(p.est + i, x0);
  S<NT>(p.est + B + i, x1);
  S<NT>(p.tru + i, x2);
  S<NT>(p.tru + B + i, x3);
  S<NT>(p.bev + i, x4);
  S<NT>(p.bev + B + i, u);
}

// two consecutive auctions per lane: 16-B f64 accesses, 8-B int32 pairs, 2-B outcome pairs
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void two(const Ptrs &p, int64_t B, int64_t i) {
  auto L2 = [&](const double *q) { return __builtin_nontemporal_load(reinterpret_cast<const f64x2 *>(q)); };
  auto S2 = [&](double *q, f64x2 v) { __builtin_nontemporal_store(v, reinterpret_cast<f64x2 *>(q)); };
  f64x2 x0 = L2(p.ctx + i), x1 = L2(p.ctx + B + i), x2 = L2(p.ctx + 2 * B + i), x3 = L2(p.ctx + 3 * B + i),
        x4 = L2(p.ctx + 4 * B + i);
  i32x2 a0 = __builtin_nontemporal_load(reinterpret_cast<const i32x2 *>(p.part + i));
  i32x2 a1 = __builtin_nontemporal_load(reinterpret_cast<const i32x2 *>(p.part + B + i));
  f64x2 u = L2(p.u + i);
  f64x2 s = x0 + x1 + x2 + x3 + x4;
  __builtin_nontemporal_store(i32x2{a0.x > a1.x, a0.y > a1.y}, reinterpret_cast<i32x2 *>(p.winner + i));
  S2(p.price + i, s * u);
  __builtin_nontemporal_store((uint16_t)((u.x > 0.5) | ((u.y > 0.5) << 8)), reinterpret_cast<uint16_t *>(p.outcome + i));
  __builtin_nontemporal_store(a0, reinterpret_cast<i32x2 *>(p.item + i));
  __builtin_nontemporal_store(a1, reinterpret_cast<i32x2 *>(p.item + B + i));
  S2(p.bid + i, s);
  S2(p.bid + B + i, s + u);
  S2(p.est + i, x0);
  S2(p.est + B + i, x1);
  S2(p.tru + i, x2);
  S2(p.tru + B + i, x3);
  S2(p.bev + i, x4);
  S2(p.bev + B + i, u);
}
__global__ __launch_bounds__(256) void k_floor_w2(Ptrs p, int64_t B) {
  for (int64_t i = 2 * ((int64_t)blockIdx.x * 256 + threadIdx.x); i < B; i += 2 * (int64_t)gridDim.x * 256) two(p, B, i);
}

__global__ __launch_bounds__(256) void k_floor_persistent(Ptrs p, int64_t B) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < B; i += (int64_t)gridDim.x * 256) one(p, B, i);
}
__global__ __launch_bounds__(256) void k_floor_persistent_nt(Ptrs p, int64_t B) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < B; i += (int64_t)gridDim.x * 256) one<true>(p, B, i);
}
__global__ __launch_bounds__(256) void k_floor_persistent_nt_wo(Ptrs p, int64_t B) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < B; i += (int64_t)gridDim.x * 256)
    one<true, true>(p, B, i);
}
__global__ __launch_bounds__(256) void k_floor_tiles(Ptrs p, int64_t B) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < B) one(p, B, i);
}


// Tiled ("AoSoA") batch layouts, 64 auctions per tile, every field of a tile contiguous:
// inputs [T][ctx0..4, u, part0|part1][64] (7 x 512 B = 3.5 KB per tile), outputs
// [T][winner|outcome (256 B), price, item0|item1, bid0, bid1, est0, est1, tru0, tru1, bev0, bev1][64]
// (84 B x 64 = 5376 B per tile): one read stream and one write stream.
template <bool TIN, bool TOUT>
__device__ __forceinline__ void one_tiled(const Ptrs &p, int64_t B, int64_t i) {
  const int64_t t = i >> 6, l = i & 63;
  double x0, x1, x2, x3, x4, u;
  int a0, a1;
  if constexpr (TIN) {
    const double *tin = p.ctx + t * 7 * 64 + l;
    x0 = __builtin_nontemporal_load(tin);
    x1 = __builtin_nontemporal_load(tin + 64);
    x2 = __builtin_nontemporal_load(tin + 128);
    x3 = __builtin_nontemporal_load(tin + 192);
    x4 = __builtin_nontemporal_load(tin + 256);
    u = __builtin_nontemporal_load(tin + 320);
    const i32x2 a = __builtin_nontemporal_load(reinterpret_cast<const i32x2 *>(tin + 384));
    a0 = a.x;
    a1 = a.y;
  } else {
    x0 = L<true>(p.ctx + i); x1 = L<true>(p.ctx + B + i); x2 = L<true>(p.ctx + 2 * B + i);
    x3 = L<true>(p.ctx + 3 * B + i); x4 = L<true>(p.ctx + 4 * B + i);
    a0 = L<true>(p.part + i); a1 = L<true>(p.part + B + i);
    u = L<true>(p.u + i);
  }
  const double s = x0 + x1 + x2 + x3 + x4;
  const int32_t wo = (int32_t)((uint32_t)(a0 > a1) | ((uint32_t)(u > 0.5) << 31));
  if constexpr (TOUT) {
    unsigned char *to = reinterpret_cast<unsigned char *>(p.price) + t * 84 * 64;
    __builtin_nontemporal_store(wo, reinterpret_cast<int32_t *>(to) + l);
    double *d = reinterpret_cast<double *>(to + 256);
    __builtin_nontemporal_store(s * u, d + l);
    __builtin_nontemporal_store(i32x2{a0, a1}, reinterpret_cast<i32x2 *>(d + 64) + l);
    __builtin_nontemporal_store(s, d + 128 + l);
    __builtin_nontemporal_store(s + u, d + 192 + l);
    __builtin_nontemporal_store(x0, d + 256 + l);
    __builtin_nontemporal_store(x1, d + 320 + l);
    __builtin_nontemporal_store(x2, d + 384 + l);
    __builtin_nontemporal_store(x3, d + 448 + l);
    __builtin_nontemporal_store(x4, d + 512 + l);
    __builtin_nontemporal_store(u, d + 576 + l);
  } else {
    S<true>(p.winner + i, wo);
    S<true>(p.price + i, s * u);
    S<true>(p.item + i, (int32_t)a0);
    S<true>(p.item + B + i, (int32_t)a1);
    S<true>(p.bid + i, s);
    S<true>(p.bid + B + i, s + u);
    S<true>(p.est + i, x0);
    S<true>(p.est + B + i, x1);
    S<true>(p.tru + i, x2);
    S<true>(p.tru + B + i, x3);
    S<true>(p.bev + i, x4);
    S<true>(p.bev + B + i, u);
  }
}
template <bool TIN, bool TOUT>
__global__ __launch_bounds__(256) void k_floor_tiled(Ptrs p, int64_t B) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < B; i += (int64_t)gridDim.x * 256)
    one_tiled<TIN, TOUT>(p, B, i);
}

// 16-B tiles: inputs [T][{x0,x1},{x2,x3},{x4,u}][64] (3 KB) + [T][part0|part1][64] (512 B);
// outputs [T][{price,bid0},{bid1,est0},{est1,tru0},{tru1,bev0},{bev1,item0|item1}][64] (5 KB)
// + [T][winner|outcome][64] (256 B): every lane access 16 B except the part pair and the word.
__global__ __launch_bounds__(256) void k_floor_tiled16(Ptrs p, int64_t B) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < B; i += (int64_t)gridDim.x * 256) {
    const int64_t t = i >> 6, l = i & 63;
    const f64x2 *tin = reinterpret_cast<const f64x2 *>(p.ctx + t * 7 * 64) + l;
    const f64x2 c0 = __builtin_nontemporal_load(tin), c1 = __builtin_nontemporal_load(tin + 64),
                c2 = __builtin_nontemporal_load(tin + 128);
    const i32x2 a = __builtin_nontemporal_load(reinterpret_cast<const i32x2 *>(p.ctx + t * 7 * 64 + 384) + l);
    const double u = c2.y;
    const double s = c0.x + c0.y + c1.x + c1.y + c2.x;
    const int32_t wo = (int32_t)((uint32_t)(a.x > a.y) | ((uint32_t)(u > 0.5) << 31));
    unsigned char *to = reinterpret_cast<unsigned char *>(p.price) + t * 84 * 64;
    f64x2 *d = reinterpret_cast<f64x2 *>(to) + l;
    __builtin_nontemporal_store(f64x2{s * u, s}, d);
    __builtin_nontemporal_store(f64x2{s + u, c0.x}, d + 64);
    __builtin_nontemporal_store(f64x2{c0.y, c1.x}, d + 128);
    __builtin_nontemporal_store(f64x2{c1.y, c2.x}, d + 192);
    __builtin_nontemporal_store(f64x2{u, __builtin_bit_cast(double, a)}, d + 256);
    __builtin_nontemporal_store(wo, reinterpret_cast<int32_t *>(to + 80 * 64) + l);
  }
}

// one tile per block, NT, the winner|outcome word: the headline's pattern in dispatch order
__global__ __launch_bounds__(256) void k_floor_tiles_nt_wo(Ptrs p, int64_t B) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < B) one<true, true>(p, B, i);
}
// persistent blocks taking 256-auction tiles from per-XCD work counters (block b counts as XCD
// b % 8, the dispatcher's round-robin): XCD x's k-th claim is tile 8 k + x, so the tiles in
// flight stay a narrow window in address order however the blocks drift. The claim for the
// next tile is made while the current one is processed.
__global__ __launch_bounds__(256) void k_floor_queue(Ptrs p, int64_t B, unsigned *ctr) {
  __shared__ unsigned s_next[2];
  const unsigned x = blockIdx.x & 7;
  const int64_t tiles = (B + 255) / 256;
  if (threadIdx.x == 0) s_next[0] = atomicAdd(ctr + 32 * x, 1u);
  __syncthreads();
  for (int k = 0;; k ^= 1) {
    const int64_t t = (int64_t)s_next[k] * 8 + x;
    if (t >= tiles) break;
    if (threadIdx.x == 0) s_next[k ^ 1] = atomicAdd(ctr + 32 * x, 1u);
    const int64_t i = t * 256 + threadIdx.x;
    if (i < B) one<true, true>(p, B, i);
    __syncthreads();
  }
}

// T consecutive tiles per block (dispatch order still follows addresses; the per-block setup
// of a real kernel is paid once per T tiles)
__global__ __launch_bounds__(256) void k_floor_chunk(Ptrs p, int64_t B, int T) {
  for (int k = 0; k < T; ++k) {
    const int64_t i = ((int64_t)blockIdx.x * T + k) * 256 + threadIdx.x;
    if (i < B) one<true, true>(p, B, i);
  }
}
extern "C" int floor_chunk(int T, const Ptrs *p, int64_t B, void *stream) {
  const int64_t tiles = (B + 255) / 256;
  hipLaunchKernelGGL(k_floor_chunk, dim3((unsigned)((tiles + T - 1) / T)), dim3(256), 0, (hipStream_t)stream, *p, B, T);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int floor_queue(int grid, const Ptrs *p, int64_t B, unsigned *ctr, void *stream) {
  hipMemsetAsync(ctr, 0, 8 * 32 * sizeof(unsigned), (hipStream_t)stream);
  hipLaunchKernelGGL(k_floor_queue, dim3(grid), dim3(256), 0, (hipStream_t)stream, *p, B, ctr);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int floor_run(int persistent, int grid, const Ptrs *p, int64_t B, void *stream) {
  if (persistent == 9) {
    hipLaunchKernelGGL(k_floor_tiles_nt_wo, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream, *p, B);
  } else if (persistent == 8) {
    hipLaunchKernelGGL(k_floor_tiled16, dim3(grid), dim3(256), 0, (hipStream_t)stream, *p, B);
  } else if (persistent >= 5 && persistent <= 7) {
    auto k = persistent == 5 ? k_floor_tiled<true, false> : persistent == 6 ? k_floor_tiled<false, true>
                                                                            : k_floor_tiled<true, true>;
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, (hipStream_t)stream, *p, B);
  } else if (persistent == 4)
    hipLaunchKernelGGL(k_floor_persistent_nt_wo, dim3(grid), dim3(256), 0, (hipStream_t)stream, *p, B);
  else if (persistent == 3)
    hipLaunchKernelGGL(k_floor_w2, dim3(grid), dim3(256), 0, (hipStream_t)stream, *p, B);
  else if (persistent == 2)
    hipLaunchKernelGGL(k_floor_persistent_nt, dim3(grid), dim3(256), 0, (hipStream_t)stream, *p, B);
  else if (persistent)
    hipLaunchKernelGGL(k_floor_persistent, dim3(grid), dim3(256), 0, (hipStream_t)stream, *p, B);
  else
    hipLaunchKernelGGL(k_floor_tiles, dim3((B + 255) / 256), dim3(256), 0, (hipStream_t)stream, *p, B);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// copy variants (the measured HBM peak): 16 B per lane
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <bool NT>
__global__ __launch_bounds__(256) void k_copy_persist(const u32x4 *src, u32x4 *dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    if constexpr (NT) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
    else dst[i] = src[i];
  }
}
template <bool NT>
__global__ __launch_bounds__(256) void k_copy_tiles(const u32x4 *src, u32x4 *dst, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    if constexpr (NT) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
    else dst[i] = src[i];
  }
}
extern "C" int copy_run(int variant, int grid, const void *src, void *dst, int64_t nbytes, void *stream) {
  const int64_t n = nbytes / 16;
  const u32x4 *s = (const u32x4 *)src;
  u32x4 *d = (u32x4 *)dst;
  hipStream_t st = (hipStream_t)stream;
  switch (variant) {
    case 0: hipLaunchKernelGGL(k_copy_persist<false>, dim3(grid), dim3(256), 0, st, s, d, n); break;
    case 1: hipLaunchKernelGGL(k_copy_persist<true>, dim3(grid), dim3(256), 0, st, s, d, n); break;
    case 2: hipLaunchKernelGGL(k_copy_tiles<false>, dim3((n + 255) / 256), dim3(256), 0, st, s, d, n); break;
    case 3: hipLaunchKernelGGL(k_copy_tiles<true>, dim3((n + 255) / 256), dim3(256), 0, st, s, d, n); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
