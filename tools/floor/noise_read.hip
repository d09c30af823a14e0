// Diagnostic: reading the Thompson noise (60 floats per (slot, auction), SP_Truthful_TS shape)
// in the ABI's tile layout -- coefficient c of auction i at ((tile)*60 + c)*64 + i%64, one
// dword per lane per coefficient (a 256-B row per wave instruction) -- against quad tiles
// (4 consecutive coefficients of an auction together: 16-B loads, a 1-KB row per wave
// instruction), each summed with trivial arithmetic so the time is the memory system's.
// Groups of G coefficients are loaded together then summed (the kernel's kTsGroup pattern).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int G>
__global__ __launch_bounds__(256) void k_rows(const float *nz, int64_t tiles, float *out) {
  for (int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); t < tiles; t += (int64_t)gridDim.x * 4) {
    const float *p = nz + t * 60 * 64 + (threadIdx.x & 63);
    float acc = 0.0f;
    for (int c0 = 0; c0 < 60; c0 += G) {
      float v[G];
#pragma unroll
      for (int g = 0; g < G; ++g) v[g] = p[(c0 + g) * 64];
#pragma unroll
      for (int g = 0; g < G; ++g) acc = acc * 0.5f + v[g];
    }
    out[t * 64 + (threadIdx.x & 63)] = acc;
  }
}
template <int G>
__global__ __launch_bounds__(256) void k_quads(const float *nz, int64_t tiles, float *out) {
  for (int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); t < tiles; t += (int64_t)gridDim.x * 4) {
    const f32x4 *p = reinterpret_cast<const f32x4 *>(nz + t * 60 * 64) + (threadIdx.x & 63);
    float acc = 0.0f;
    for (int q0 = 0; q0 < 15; q0 += G) {
      f32x4 v[G];
#pragma unroll
      for (int g = 0; g < G; ++g) v[g] = q0 + g < 15 ? p[(q0 + g) * 64] : f32x4{0, 0, 0, 0};
#pragma unroll
      for (int g = 0; g < G; ++g) acc = ((acc * 0.5f + v[g].x) + v[g].y) + (v[g].z + v[g].w);
    }
    out[t * 64 + (threadIdx.x & 63)] = acc;
  }
}

extern "C" int noise_run(int variant, int grid, const float *nz, int64_t tiles, float *out, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  switch (variant) {
    case 0: hipLaunchKernelGGL(k_rows<20>, dim3(grid), dim3(256), 0, st, nz, tiles, out); break;
    case 1: hipLaunchKernelGGL(k_rows<60>, dim3(grid), dim3(256), 0, st, nz, tiles, out); break;
    case 2: hipLaunchKernelGGL(k_quads<5>, dim3(grid), dim3(256), 0, st, nz, tiles, out); break;
    case 3: hipLaunchKernelGGL(k_quads<15>, dim3(grid), dim3(256), 0, st, nz, tiles, out); break;
    case 4: hipLaunchKernelGGL(k_rows<4>, dim3(grid), dim3(256), 0, st, nz, tiles, out); break;
    case 5: hipLaunchKernelGGL(k_quads<1>, dim3(grid), dim3(256), 0, st, nz, tiles, out); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
