"""The kernels' exp (auction-gym_amd/csrc/ag_exp.h) compiled for the HOST from the very
same source, against the host glibc exp, bit for bit, over 4e7 inputs covering the whole
double range (the device build is compared with libm in tests/test_gpu_parity.py)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

SRC = r'''
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include "ag_exp.h"
#include "ag_exp_table.h"
static unsigned long long s = 88172645463325252ull;
static inline unsigned long long xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
int main(int argc, char **argv) {
  long n = atol(argv[1]), bad = 0, sbad = 0;
  for (long i = 0; i < n; ++i) {
    double x; int m = i % 5;
    if (m == 0) x = (double)(xr() >> 11) * 0x1p-53 * 100 - 50;
    else if (m == 1) x = (double)(xr() >> 11) * 0x1p-53 * 1460 - 750;
    else if (m == 2) x = (double)(xr() >> 11) * 0x1p-53 * 16 - 8;
    else if (m == 3) x = (double)(xr() >> 11) * 0x1p-53 * 0x1p-40;
    else { unsigned long long u = xr(); __builtin_memcpy(&x, &u, 8); }
    if (x != x) continue;
    double a = exp(x), b = agexp::exp(x, ag_exp_tab);
    if (__builtin_memcmp(&a, &b, 8)) { if (bad < 5) printf("x=%a libm=%a mine=%a\n", x, a, b); bad++; }
    double sa = 1.0 / (1.0 + exp(-x)), sb = agexp::sigmoid(x, ag_exp_tab);
    if (__builtin_memcmp(&sa, &sb, 8)) sbad++;
  }
  printf("bad %ld sbad %ld of %ld\n", bad, sbad, n);
  return bad || sbad;
}
'''


def test_host_build_of_device_exp_matches_glibc(tmp_path):
    c = tmp_path / "t.cpp"
    c.write_text(SRC)
    exe = tmp_path / "t"
    inc = os.path.join(ROOT, "auction-gym_amd", "csrc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", inc, str(c), "-o", str(exe),
                    "-lm"], check=True)
    r = subprocess.run([str(exe), "40000000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout


EXPF_SRC = r'''
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include "ag_exp.h"
#include "ag_exp_table.h"
static long bad = 0, n = 0;
static uint64_t tab32[32];
static void check(unsigned b) {
  float x; memcpy(&x, &b, 4); ++n;
  float a = expf(x), m = agexp::expf_glibc(x, tab32);
  if (isnan(a) && isnan(m)) return;
  if (memcmp(&a, &m, 4)) { if (bad < 5) printf("x=%a libm=%a mine=%a\n", x, a, m); ++bad; }
}
int main(int argc, char **argv) {
  unsigned stride = (unsigned)atoi(argv[1]), off = (unsigned)atoi(argv[2]);
  for (int j = 0; j < 32; ++j) tab32[j] = agexp::expf_tab_entry(ag_exp_tab, j);
  for (unsigned long long u = off; u < (1ull << 32); u += stride) check((unsigned)u);
  /* the range edges: +-0, +-inf, nan, around 88 / 88.72 / -103.28 / -103.97 / -104 */
  const unsigned edge[] = {0u, 0x80000000u, 0x7f800000u, 0xff800000u, 0x7fc00000u, 0xffc00000u};
  for (unsigned e : edge) check(e);
  const unsigned mid[] = {0x42b00000u, 0x42b17218u, 0xc2ce8ed0u, 0xc2cff1b4u, 0xc2d00000u, 0xc2b00000u};
  for (unsigned c : mid) for (int d = -64; d <= 64; ++d) check(c + d);
  printf("bad %ld of %ld\n", bad, n);
  return bad != 0;
}
'''


def test_host_build_of_device_expf_matches_glibc(tmp_path):
    """agexp::expf_glibc (torch.sigmoid's scalar path, the LR-TS CTRs) against the host libm
    expf: every 7th float bit pattern (a sixth of a billion, all exponents and signs) plus
    the range edges (+-0, +-inf, nan, the overflow / underflow thresholds). The full 2^32
    sweep (stride 1) also passes; it takes ~90 s, so the suite runs the strided one."""
    c = tmp_path / "f.cpp"
    c.write_text(EXPF_SRC)
    exe = tmp_path / "f"
    inc = os.path.join(ROOT, "auction-gym_amd", "csrc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", inc, str(c), "-o", str(exe),
                    "-lm"], check=True)
    r = subprocess.run([str(exe), "7", "3"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout


def test_log1p_restatement_accuracy():
    """The fdlibm log1p the DR bidder's softplus uses (oracle/ag_oracle_dr.c; the device's
    csrc/ag_log1p.h is the same algorithm): within 1 ulp of libm over its whole use range."""
    import math
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    L = O.lib()
    g = np.random.default_rng(0)
    xs = np.concatenate([np.exp(g.uniform(-40, 20, 100000)), g.uniform(-0.99, 1, 50000),
                         [0.0, 1e-300, 1e-20, 0.4142135, -0.29289, 1e300, 2.0 ** -29, 2.0 ** -54]])
    worst = 0.0
    for x in xs:
        a, b = L.ora_log1p_restated(float(x)), math.log1p(x)
        if a != b:
            worst = max(worst, abs(a - b) / abs(b))
    assert worst < 2.3e-16


MAIN_SRC = r'''
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include "ag_exp.h"
#include "ag_exp_table.h"
#include "ag_log1p.h"
static unsigned long long s = 88172645463325252ull;
static inline unsigned long long xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
int main(int argc, char **argv) {
  long n = atol(argv[1]), ebad = 0, lbad = 0, eok = 0, lok = 0;
  for (long i = 0; i < n; ++i) {
    double x; int m = i % 6;
    if (m == 0) x = (double)(xr() >> 11) * 0x1p-53 * 100 - 50;
    else if (m == 1) x = (double)(xr() >> 11) * 0x1p-53 * 1460 - 750;
    else if (m == 2) x = (double)(xr() >> 11) * 0x1p-53 * 16 - 8;
    else if (m == 3) x = ldexp((double)(xr() >> 11) * 0x1p-53 + 0.5, (int)(xr() % 120) - 60);
    else if (m == 4) x = (double)(xr() >> 11) * 0x1p-53 * 3;
    else { unsigned long long u = xr(); __builtin_memcpy(&x, &u, 8); }
    if (x != x) continue;
    if (agexp::exp_in_main(x)) {
      ++eok;
      double a = agexp::exp(x, ag_exp_tab), b = agexp::exp_main(x, ag_exp_tab);
      if (__builtin_memcmp(&a, &b, 8)) { if (ebad < 5) printf("exp x=%a %a %a\n", x, a, b); ebad++; }
    }
    double y = fabs(x);
    bool ok;
    double lb = aglog1p::log1p_main(y, ok);
    if (ok) {
      ++lok;
      double la = aglog1p::log1p(y);
      if (__builtin_memcmp(&la, &lb, 8)) { if (lbad < 5) printf("log1p x=%a %a %a\n", y, la, lb); lbad++; }
    }
  }
  printf("exp bad %ld of %ld; log1p bad %ld of %ld\n", ebad, eok, lbad, lok);
  return ebad || lbad;
}
'''


def test_branch_free_main_paths_match(tmp_path):
    """agexp::exp_main / aglog1p::log1p_main (the trainer's branch-free fast paths) equal
    agexp::exp / aglog1p::log1p bit for bit wherever they report themselves valid, over
    3e7 inputs (whole double range, the softplus range, powers of two 2^-60..2^60)."""
    c = tmp_path / "m.cpp"
    c.write_text(MAIN_SRC)
    exe = tmp_path / "m"
    inc = os.path.join(ROOT, "auction-gym_amd", "csrc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", inc, str(c), "-o", str(exe),
                    "-lm"], check=True)
    r = subprocess.run([str(exe), "30000000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout
