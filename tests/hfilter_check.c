// Test helper (not product): host restatement of the scaled packed-fp32
// homography filter (verify_kernels.hip: h_filter_consts / h_filter_pair) on
// random homographies and points placed near the decision boundary; checks
// that every decided point agrees with the fp64 reference residual and
// reports the undecided fraction.
// build: gcc -O2 -ffp-contract=off -o hfc tests/hfilter_check.c -lm (tests/test_filter_bounds.py)
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static double urand(uint64_t* s) {
  *s = *s * 6364136223846793005ull + 1442695040888963407ull;
  return (double)(*s >> 11) * 0x1p-53;
}

static float f_ru(double v) {  // round toward +inf
  float f = (float)v;
  if ((double)f < v) f = nextafterf(f, INFINITY);
  return f;
}

static void consts(const double* H, double S, double maxr, float* c) {
  const double u = 0x1p-24, r = 1.0 / sqrt(maxr);
  double Hs[9];
  for (int j = 0; j < 6; ++j) Hs[j] = H[j] * r;
  for (int j = 6; j < 9; ++j) Hs[j] = H[j];
  const double A0 = (fabs(Hs[0]) + fabs(Hs[1])) * S + fabs(Hs[2]);
  const double A1 = (fabs(Hs[3]) + fabs(Hs[4])) * S + fabs(Hs[5]);
  const double A2 = (fabs(Hs[6]) + fabs(Hs[7])) * S + fabs(Hs[8]);
  const double al0 = 3.01 * u * A0, al1 = 3.01 * u * A1, al2 = 3.01 * u * A2;
  const double b = S * r * (1.0001 * al2 + 2.02 * u * A2) + fmax(al0, al1);
  const double E = (2.85 * b + 2.0 * al2) * A2 + 6.1 * b * b + al2 * al2 + 5.2 * u * A2 * A2;
  for (int j = 0; j < 9; ++j) c[j] = (float)Hs[j];
  c[9] = f_ru(1.5 * E + 1e-30);
}

// The previous filter (per-point margin a2 maxr Q2^2 + a0, unscaled points).
static void consts_old(const double* H, double S, double maxr, float* c) {
  const double u = 0x1p-24;
  const double A0 = (fabs(H[0]) + fabs(H[1])) * S + fabs(H[2]);
  const double A1 = (fabs(H[3]) + fabs(H[4])) * S + fabs(H[5]);
  const double A2 = (fabs(H[6]) + fabs(H[7])) * S + fabs(H[8]);
  const double al0 = 3.01 * u * A0, al1 = 3.01 * u * A1, al2 = 3.01 * u * A2;
  const double b = S * al2 + fmax(al0, al1);
  const double sq = sqrt(maxr);
  const double c1 = 2.0 * maxr * al2 + 2.85 * b * sq;
  const double c0 = 3.0 * maxr * al2 * al2 + 2.85 * b * sq * al2 + 2.01 * b * b;
  double tau = fabs(H[6] * (0.5 * S) + H[7] * (0.5 * S) + H[8]);
  if (!(tau > 1e-30 && tau < 1e30)) tau = A2 > 1e-30 ? A2 : 1e-30;
  const double a2 = 1.5 * (7.2 * u + 1.01 * c1 / (2.0 * tau * maxr));
  const double a0 = 1.5 * (c0 + 0.5 * c1 * tau) + 1e-30;
  for (int j = 0; j < 9; ++j) c[j] = (float)H[j];
  c[9] = f_ru(a0);
  c[10] = f_ru(a2 * maxr);
}

static double ref_res(const double* H, double s0, double s1, double d0, double d1) {
  const double p0 = H[0] * s0 + H[1] * s1 + H[2];
  const double p1 = H[3] * s0 + H[4] * s1 + H[5];
  const double p2 = H[6] * s0 + H[7] * s1 + H[8];
  const double inv = 1.0 / p2;
  const double dd0 = d0 - p0 * inv, dd1 = d1 - p1 * inv;
  return dd0 * dd0 + dd1 * dd1;
}

int main(int argc, char** argv) {
  const double maxr = argc > 1 ? atof(argv[1]) : 16.0;
  const float ds = (float)(1.0 / sqrt(maxr));
  uint64_t seed = 12345;
  const int uni = argc > 2;  // uniform radii in [0, 3 sqrt(maxr)]
  long n = 0, und = 0, bad = 0, inl = 0, und_old = 0;
  for (int m = 0; m < 20000; ++m) {
    double H[9];
    const double S = 200.0 + 3000.0 * urand(&seed);
    const double th = 0.3 * (urand(&seed) - 0.5), sc = 0.7 + 0.6 * urand(&seed);
    H[0] = sc * cos(th) + 0.05 * (urand(&seed) - 0.5);
    H[1] = -sc * sin(th) + 0.05 * (urand(&seed) - 0.5);
    H[2] = 200.0 * (urand(&seed) - 0.5);
    H[3] = sc * sin(th) + 0.05 * (urand(&seed) - 0.5);
    H[4] = sc * cos(th) + 0.05 * (urand(&seed) - 0.5);
    H[5] = 200.0 * (urand(&seed) - 0.5);
    H[6] = 2e-4 * (urand(&seed) - 0.5);
    H[7] = 2e-4 * (urand(&seed) - 0.5);
    H[8] = 0.5 + urand(&seed);
    const double k = 1.0 / sqrt(H[0] * H[0] + H[4] * H[4] + H[8] * H[8]);  // arbitrary scale
    for (int j = 0; j < 9; ++j) H[j] *= k * (0.01 + 100.0 * urand(&seed));
    float c[10], co[11];
    consts(H, S, maxr, c);
    consts_old(H, S, maxr, co);
    for (int p = 0; p < 400; ++p) {
      const float s0 = (float)(S * urand(&seed)), s1 = (float)(S * urand(&seed));
      const double p0 = H[0] * s0 + H[1] * s1 + H[2], p1 = H[3] * s0 + H[4] * s1 + H[5];
      const double p2 = H[6] * s0 + H[7] * s1 + H[8];
      // destination near the boundary: radius sqrt(maxr) * (1 +- tiny) around the transfer
      const double ang = 6.283185307179586 * urand(&seed);
      const double rad = sqrt(maxr) * (1.0 + (p & 1 ? 1e-7 : 1e-3) * (2.0 * urand(&seed) - 1.0)) *
                         (uni || p % 7 == 0 ? urand(&seed) * 3.0 : 1.0);
      const float d0 = (float)(p0 / p2 + rad * cos(ang)), d1 = (float)(p1 / p2 + rad * sin(ang));
      if (fabsf(d0) > S || fabsf(d1) > S) continue;
      const float dd0 = d0 * ds, dd1 = d1 * ds;
      const float t0 = fmaf(c[1], s1, c[2]), t1 = fmaf(c[4], s1, c[5]), t2 = fmaf(c[7], s1, c[8]);
      const float q0 = fmaf(c[0], s0, t0), q1 = fmaf(c[3], s0, t1), q2 = fmaf(c[6], s0, t2);
      const float w0 = fmaf(dd0, q2, -q0), w1 = fmaf(dd1, q2, -q1);
      const float lhs = fmaf(w0, w0, w1 * w1);
      const float diff = fmaf(-q2, q2, lhs);
      const int in_ref = ref_res(H, s0, s1, d0, d1) <= maxr;
      {
        const float T0 = fmaf(co[1], s1, co[2]), T1 = fmaf(co[4], s1, co[5]), T2 = fmaf(co[7], s1, co[8]);
        const float Q0 = fmaf(co[0], s0, T0), Q1 = fmaf(co[3], s0, T1), Q2 = fmaf(co[6], s0, T2);
        const float W0 = fmaf(d0, Q2, -Q0), W1 = fmaf(d1, Q2, -Q1);
        const float L = fmaf(W0, W0, W1 * W1), qq = Q2 * Q2;
        const float mg = fmaf(co[10], qq, co[9]);
        const float df = fmaf(-(float)maxr, qq, L);
        und_old += fabsf(df) <= mg;
      }
      ++n;
      inl += in_ref;
      if (fabsf(diff) <= c[9]) {
        ++und;
      } else if ((diff < -c[9]) != in_ref) {
        ++bad;
        if (bad < 5) printf("BAD m=%d diff=%g M=%g ref=%d\n", m, diff, c[9], in_ref);
      }
    }
  }
  printf("maxr=%g points=%ld inliers=%ld undecided=%ld (%.4f%%; previous filter %.4f%%) wrong=%ld\n",
         maxr, n, inl, und, 100.0 * und / n, 100.0 * und_old / n, bad);
  return bad != 0;
}
