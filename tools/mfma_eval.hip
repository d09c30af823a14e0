// mfma_eval.hip -- MFMA vs VALU for the learners' win-rate fit (north star: "MFMA used only
// for the small MLP value/CTR forward+backward"). Standalone measurement, not
// part of the library.
//
// The fit (src/Models.py:51-62 PyTorchWinRateEstimator, the loop of src/Bidder.py:517-538;
// auction-gym_amd/csrc/ag_dr.hip fit_winrate) is, per record and epoch, two BCE rows of a
// 4-wide linear model: z = [c v g 1] . w, p = sigmoid(z), loss softplus(+-z), and the
// gradient terms (p - y) [c v g 1]. As matrices: Z = X w (X [n][4], w [4][1]) and
// grad = X^T (p - y) -- a GEMV with K = 4 and a reduction with M = 4. Two ways to run them
// over records staged in LDS (as the trainer stages them), the same transcendental work
// per row in both (exp, log1p, reciprocal: the part the model's width does not change):
//   VALU: one record per lane, z by 3 FP64 mul + 3 add, gradient terms by 4 FP64 mul/adds
//         into per-lane accumulators;
//   MFMA: v_mfma_f64_16x16x4_f64 -- forward: A = 16 records x 4 features, B = w replicated
//         over the 16 columns, so 4 MFMAs give 64 records' z (brought to one record per lane
//         with one ds_bpermute pair each); backward: A = 16 (4 useful) features x 4
//         records, B = 4 records' (p - y) over the 16 columns, accumulated over the records:
//         16 MFMAs per 64 records.
// Both compute the same values; the kernels report (checksums) and the host prints the
// time per epoch. Modes: 0 = full rows, 1 = contraction only (no transcendentals).
//
//   hipcc --offload-arch=gfx950 -O3 -o build/mfma_eval tools/mfma_eval.hip && build/mfma_eval
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int kT = 256;
constexpr int kRec = 4096;  // records per workgroup, staged in LDS as [rec][c v g y] float

__device__ __forceinline__ double bperm(double x, int src_lane) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_ds_bpermute(src_lane * 4, (int)(b & 0xffffffff));
  const int hi = __builtin_amdgcn_ds_bpermute(src_lane * 4, (int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// the per-row work that does not depend on how z was formed: loss and p - y
template <int MODE>
__device__ __forceinline__ void row_tail(double z, double y, double &loss, double &gz) {
  if (MODE == 0) {
    const double em = exp(-z);
    const double u = y > 0.0 ? -z : z;
    const double eu = y > 0.0 ? em : exp(z);
    loss += u > 20.0 ? u : log1p(eu);
    gz = 1.0 / (1.0 + em) - y;
  } else {
    loss += z;
    gz = z * 0.25 - y;
  }
}

template <int MODE>
__global__ __launch_bounds__(kT) void k_valu(const float4 *__restrict__ rec, int epochs, const double *w0,
                                           double *out) {
  __shared__ float4 s[kRec];
  const float4 *r = rec + (size_t)blockIdx.x * kRec;
  for (int i = threadIdx.x; i < kRec; i += kT) s[i] = r[i];
  __syncthreads();
  double w[4] = {w0[0], w0[1], w0[2], w0[3]};
  double tot = 0.0;
  for (int e = 0; e < epochs; ++e) {
    double acc[5] = {0, 0, 0, 0, 0};
    for (int j = threadIdx.x; j < kRec; j += kT) {
      const float4 q = s[j];
      const double c = q.x, v = q.y, g = q.z, y = q.w;
      for (int aug = 0; aug < 2; ++aug) {  // the logged row, then gamma = 0, y = 0
        const double gg = aug ? 0.0 : g, yy = aug ? 0.0 : y;
        const double z = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(c, w[0]), __dmul_rn(v, w[1])),
                                             __dmul_rn(gg, w[2])), w[3]);
        double gz;
        row_tail<MODE>(z, yy, acc[0], gz);
        acc[1] += gz * c;
        acc[2] += gz * v;
        acc[3] += gz * gg;
        acc[4] += gz;
      }
    }
    // the step the trainer takes after its block/agent sums (here: per lane, to keep the
    // epochs dependent without a barrier)
    for (int k = 0; k < 4; ++k) w[k] -= 1e-9 * acc[1 + k];
    tot += acc[0];
  }
  out[blockIdx.x * kT + threadIdx.x] = tot + w[0] + w[1] + w[2] + w[3];
}

template <int MODE>
__global__ __launch_bounds__(kT) void k_mfma(const float4 *__restrict__ rec, int epochs, const double *w0,
                                           double *out) {
  __shared__ float4 s[kRec];
  const float4 *r = rec + (size_t)blockIdx.x * kRec;
  for (int i = threadIdx.x; i < kRec; i += kT) s[i] = r[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double w[4] = {w0[0], w0[1], w0[2], w0[3]};
  double tot = 0.0;
  const float *sf = reinterpret_cast<const float *>(s);
  for (int e = 0; e < epochs; ++e) {
    double loss = 0.0;
    f64x4 gacc = {0.0, 0.0, 0.0, 0.0};  // C of the gradient MFMAs: row = feature
    for (int base = wave * 64; base < kRec; base += kT) {
      for (int aug = 0; aug < 2; ++aug) {
        // forward: 4 MFMAs, group q = records base + 16 q .. +15
        double zl = 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int recA = base + 16 * q + (lane & 15), k = lane >> 4;  // A[rec][feature k]
          double a = k == 3 ? 1.0 : (double)sf[recA * 4 + k];
          if (aug && k == 2) a = 0.0;
          const double b = w[k];  // B[k][col] = w_k for every col
          f64x4 c = {0.0, 0.0, 0.0, 0.0};
          c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
          // C: col = lane & 15, row = (lane >> 4) + 4 reg, every column the same. Record
          // row t of the group lives in lanes (t & 3) * 16 + col, reg t >> 2: lane s sends
          // its reg (s & 3) (columns 0..3 cover every reg), the lane of record t reads lane
          // (t & 3) * 16 + (t >> 2).
          const int t = lane & 15;
          const int sr = lane & 3;
          const double mine = sr == 0 ? c[0] : sr == 1 ? c[1] : sr == 2 ? c[2] : c[3];
          const double zq = bperm(mine, (t & 3) * 16 + (t >> 2));
          if ((lane >> 4) == q) zl = zq;
        }
        const float4 qv = s[base + lane];
        const double yy = aug ? 0.0 : (double)qv.w;
        double gz;
        row_tail<MODE>(zl, yy, loss, gz);
        // backward: grad[f] = sum_rec X[rec][f] gz[rec]; 16 MFMAs of 4 records each
#pragma unroll
        for (int m = 0; m < 16; ++m) {
          const int kr = lane >> 4, f = lane & 15;   // A[row f][k = record 4m + kr]
          const int rr = base + 4 * m + kr;
          double a = f < 3 ? (double)sf[rr * 4 + f] : (f == 3 ? 1.0 : 0.0);
          if (aug && f == 2) a = 0.0;
          const double b = bperm(gz, 4 * m + kr);    // B[k = record][col] = gz of that record
          gacc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, gacc, 0, 0, 0);
        }
      }
    }
    // gradient rows 0..3 live in reg 0 of lanes 0..15 (row = lane >> 4 + 4 reg) -> rows
    // 0..3 are reg 0 of lane groups 0..3; broadcast them
    double g4[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) g4[k] = bperm(gacc[0], 16 * k);
    for (int k = 0; k < 4; ++k) w[k] -= 1e-9 * g4[k];
    tot += loss;
  }
  out[blockIdx.x * kT + threadIdx.x] = tot + w[0] + w[1] + w[2] + w[3];
}

// One wave, records 0..63 (logged rows), fixed w: z by the MFMA forward, grad by the MFMA
// backward with gz = z (no transcendentals) -- checked on the host against plain sums.
__global__ void k_check(const float4 *__restrict__ rec, const double *w, double *z_out, double *g_out) {
  const int lane = threadIdx.x;
  const float *sf = reinterpret_cast<const float *>(rec);
  double zl = 0.0;
  for (int q = 0; q < 4; ++q) {
    const int k = lane >> 4;
    const double a = k == 3 ? 1.0 : (double)sf[(16 * q + (lane & 15)) * 4 + k];
    f64x4 c = {0.0, 0.0, 0.0, 0.0};
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, w[k], c, 0, 0, 0);
    const int t = lane & 15, sr = lane & 3;
    const double mine = sr == 0 ? c[0] : sr == 1 ? c[1] : sr == 2 ? c[2] : c[3];
    const double zq = bperm(mine, (t & 3) * 16 + (t >> 2));
    if ((lane >> 4) == q) zl = zq;
  }
  z_out[lane] = zl;
  f64x4 gacc = {0.0, 0.0, 0.0, 0.0};
  for (int m = 0; m < 16; ++m) {
    const int kr = lane >> 4, f = lane & 15;
    const double a = f < 3 ? (double)sf[(4 * m + kr) * 4 + f] : (f == 3 ? 1.0 : 0.0);
    gacc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bperm(zl, 4 * m + kr), gacc, 0, 0, 0);
  }
  const double gk = bperm(gacc[0], 16 * (lane & 3));  // every lane takes part (bpermute reads
  if (lane < 4) g_out[lane] = gk;                     // only from active lanes)
}

int main(int argc, char **argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 171 * 3;  // the bench's FP_DM_TS split: 3 agents
  const int epochs = argc > 2 ? atoi(argv[2]) : 64;
  const size_t n = (size_t)blocks * kRec;
  std::vector<float> h(n * 4);
  srand(1);
  for (size_t i = 0; i < n; ++i) {
    h[4 * i] = (float)rand() / RAND_MAX;
    h[4 * i + 1] = 0.5f + (float)rand() / RAND_MAX;
    h[4 * i + 2] = (float)rand() / RAND_MAX;
    h[4 * i + 3] = (rand() & 1) ? 1.0f : 0.0f;
  }
  float4 *d;
  double *w, *o;
  CK(hipMalloc(&d, n * 16));
  CK(hipMalloc(&w, 32));
  CK(hipMalloc(&o, (size_t)blocks * kT * 8));
  CK(hipMemcpy(d, h.data(), n * 16, hipMemcpyHostToDevice));
  const double hw[4] = {0.3, -0.2, 0.7, 0.1};
  CK(hipMemcpy(w, hw, 32, hipMemcpyHostToDevice));
  {
    double *dz, *dg;
    CK(hipMalloc(&dz, 64 * 8));
    CK(hipMalloc(&dg, 4 * 8));
    hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, d, w, dz, dg);
    double hz[64], hg[4], rg[4] = {0, 0, 0, 0}, ez = 0, eg = 0;
    CK(hipMemcpy(hz, dz, sizeof hz, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hg, dg, sizeof hg, hipMemcpyDeviceToHost));
    for (int r = 0; r < 64; ++r) {
      const double x[4] = {h[4 * r], h[4 * r + 1], h[4 * r + 2], 1.0};
      double z = 0;
      for (int k = 0; k < 4; ++k) z += x[k] * hw[k];
      ez = fmax(ez, fabs(z - hz[r]) / fabs(z));
      for (int k = 0; k < 4; ++k) rg[k] += x[k] * z;
    }
    for (int k = 0; k < 4; ++k) eg = fmax(eg, fabs(rg[k] - hg[k]) / fabs(rg[k]));
    printf("MFMA layout check (64 records): max rel err z %.2e, grad %.2e\n", ez, eg);
  }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char *name, void (*k)(const float4 *, int, const double *, double *)) {
    hipLaunchKernelGGL(k, dim3(blocks), dim3(kT), 0, 0, d, 2, w, o);  // warm
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(kT), 0, 0, d, epochs, w, o);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<double> ho((size_t)blocks * kT);
    CK(hipMemcpy(ho.data(), o, ho.size() * 8, hipMemcpyDeviceToHost));
    double cs = 0;
    for (double x : ho) cs += x;
    printf("%-22s %9.3f us/epoch  %7.3f ns/record-epoch  checksum %.12e\n", name, ms * 1e3 / epochs,
           ms * 1e6 / epochs / (double)n, cs);
  };
  printf("records %zu (%d workgroups x %d), %d epochs, 2 BCE rows per record\n", n, blocks, kRec, epochs);
  run("VALU full rows", k_valu<0>);
  run("MFMA full rows", k_mfma<0>);
  run("VALU contraction only", k_valu<1>);
  run("MFMA contraction only", k_mfma<1>);
  return 0;
}
