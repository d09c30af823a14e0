#include <immintrin.h>
#include <ATen/native/cpu/avx_mathfun.h>
extern "C" void blk(float *data) {
  const __m256 two_pi = _mm256_set1_ps(2.0f * 3.14159265358979323846);
  const __m256 one = _mm256_set1_ps(1.0f), minus_two = _mm256_set1_ps(-2.0f);
  const __m256 u1 = _mm256_sub_ps(one, _mm256_loadu_ps(data));
  const __m256 u2 = _mm256_loadu_ps(data + 8);
  const __m256 radius = _mm256_sqrt_ps(_mm256_mul_ps(minus_two, log256_ps(u1)));
  const __m256 theta = _mm256_mul_ps(two_pi, u2);
  __m256 s, c;
  sincos256_ps(theta, &s, &c);
  _mm256_storeu_ps(data, _mm256_mul_ps(radius, c));
  _mm256_storeu_ps(data + 8, _mm256_mul_ps(radius, s));
}
