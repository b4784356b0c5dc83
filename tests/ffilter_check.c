// Test helper (not product): host restatement of the packed-fp32 Sampson
// inlier filter (verify_kernels.hip: f_filter_consts / f_filter_pair) on
// random fundamental matrices F = [t]x M of arbitrary scale, with second
// points placed (by bisection along the epipolar line's normal) within 1e-7 or
// 1e-3 (relative) of the threshold, or uniformly around it; checks that every
// point the filter decides agrees with the fp64 reference Sampson error
// (ComputeSquaredSampsonError) and reports the undecided share.
// build: gcc -O2 -ffp-contract=off -o ffc tests/ffilter_check.c -lm (tests/test_filter_bounds.py)
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static double urand(uint64_t* s) {
  *s = *s * 6364136223846793005ull + 1442695040888963407ull;
  return (double)(*s >> 11) * 0x1p-53;
}

static float f_ru(double v) {
  float f = (float)v;
  if ((double)f < v) f = nextafterf(f, INFINITY);
  return f;
}

static void consts(const double* F, double S, double maxr, float* c) {
  const double u = 0x1p-24;
  const double A0 = (fabs(F[0]) + fabs(F[1])) * S + fabs(F[2]);
  const double A1 = (fabs(F[3]) + fabs(F[4])) * S + fabs(F[5]);
  const double A2 = (fabs(F[6]) + fabs(F[7])) * S + fabs(F[8]);
  const double B0 = (fabs(F[0]) + fabs(F[3])) * S + fabs(F[6]);
  const double B1 = (fabs(F[1]) + fabs(F[4])) * S + fabs(F[7]);
  const double al0 = 3.01 * u * A0, al1 = 3.01 * u * A1, al2 = 3.01 * u * A2;
  const double be0 = 3.01 * u * B0, be1 = 3.01 * u * B1;
  const double g = S * (al0 + al1) + al2 + 2.01 * u * (S * (A0 + A1) + A2);
  const double d = fmax(fmax(al0, al1), fmax(be0, be1));
  const double sq = sqrt(maxr);
  const double c1 = 2.0 * g * sq + 4.0 * d * maxr;
  const double c0 = g * g + 2.0 * maxr * d * d;
  const double h = 0.5 * S;
  const double m0 = F[0] * h + F[1] * h + F[2], m1 = F[3] * h + F[4] * h + F[5];
  const double n0 = F[0] * h + F[3] * h + F[6], n1 = F[1] * h + F[4] * h + F[7];
  double tau = sqrt(m0 * m0 + m1 * m1 + n0 * n0 + n1 * n1);
  const double tmax = A0 + A1 + B0 + B1;
  if (!(tau > 1e-30 && tau < 1e30)) tau = tmax > 1e-30 ? tmax : 1e-30;
  const double a1 = 1.5 * (1.01 * c1 / (2.0 * tau * maxr) + 5.1 * u);
  const double a0 = 1.5 * (0.5 * c1 * tau + c0) + 1e-30;
  for (int j = 0; j < 9; ++j) c[j] = (float)F[j];
  c[9] = f_ru(a0);
  c[10] = f_ru(a1);
}

static double sampson(const double* F, double x0, double x1, double y0, double y1) {
  const double a0 = F[0] * x0 + F[1] * x1 + F[2], a1 = F[3] * x0 + F[4] * x1 + F[5];
  const double a2 = F[6] * x0 + F[7] * x1 + F[8];
  const double b0 = F[0] * y0 + F[3] * y1 + F[6], b1 = F[1] * y0 + F[4] * y1 + F[7];
  const double e = y0 * a0 + y1 * a1 + a2;
  return e * e / (a0 * a0 + a1 * a1 + b0 * b0 + b1 * b1);
}

int main(int argc, char** argv) {
  const double maxr = argc > 1 ? atof(argv[1]) : 16.0;
  const int uni = argc > 2;
  uint64_t seed = 777;
  long n = 0, und = 0, bad = 0, inl = 0;
  for (int m = 0; m < 3000; ++m) {
    const double S = 200.0 + 3000.0 * urand(&seed);
    double t[3], M[9], F[9];
    for (int j = 0; j < 3; ++j) t[j] = urand(&seed) - 0.5;
    t[2] *= 0.2;
    for (int j = 0; j < 9; ++j) M[j] = (j % 4 == 0 ? 1.0 : 0.0) + 0.1 * (urand(&seed) - 0.5);
    M[2] = 0.002 * (urand(&seed) - 0.5) * S;  // translations in pixels
    M[5] = 0.002 * (urand(&seed) - 0.5) * S;
    const double T[9] = {0, -t[2], t[1], t[2], 0, -t[0], -t[1], t[0], 0};
    const double k = pow(10.0, 4.0 * urand(&seed) - 2.0);  // arbitrary scale
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c)
        F[3 * r + c] = k * (T[3 * r] * M[c] + T[3 * r + 1] * M[3 + c] + T[3 * r + 2] * M[6 + c]);
    float cf[11];
    consts(F, S, maxr, cf);
    for (int p = 0; p < 300; ++p) {
      const float x0 = (float)(S * urand(&seed)), x1 = (float)(S * urand(&seed));
      // epipolar line l = F x1 in image 2; a point on it and its unit normal
      const double l0 = F[0] * x0 + F[1] * x1 + F[2], l1 = F[3] * x0 + F[4] * x1 + F[5];
      const double l2 = F[6] * x0 + F[7] * x1 + F[8];
      const double nn = sqrt(l0 * l0 + l1 * l1);
      if (!(nn > 0)) continue;
      const double ux = l0 / nn, uy = l1 / nn;
      const double foot_x = -l2 * ux / nn, foot_y = -l2 * uy / nn;
      const double along = S * (urand(&seed) - 0.5);
      const double px = foot_x - uy * along, py = foot_y + ux * along;
      double lo = 0.0, hi = 100.0 * sqrt(maxr);
      double target = maxr * (1.0 + (p & 1 ? 1e-7 : 1e-3) * (2.0 * urand(&seed) - 1.0));
      if (uni || p % 7 == 0) target = maxr * 9.0 * urand(&seed);
      for (int it = 0; it < 60; ++it) {
        const double mid = 0.5 * (lo + hi);
        if (sampson(F, x0, x1, px + mid * ux, py + mid * uy) < target) lo = mid;
        else hi = mid;
      }
      const float y0 = (float)(px + lo * ux), y1 = (float)(py + lo * uy);
      if (!(fabsf(y0) <= S && fabsf(y1) <= S)) continue;
      // the filter, as f_filter_pair evaluates one lane
      const float t0 = fmaf(cf[1], x1, cf[2]), U0 = fmaf(cf[0], x0, t0);
      const float t1 = fmaf(cf[4], x1, cf[5]), U1 = fmaf(cf[3], x0, t1);
      const float t2 = fmaf(cf[7], x1, cf[8]), U2 = fmaf(cf[6], x0, t2);
      const float t3 = fmaf(cf[3], y1, cf[6]), V0 = fmaf(cf[0], y0, t3);
      const float t4 = fmaf(cf[4], y1, cf[7]), V1 = fmaf(cf[1], y0, t4);
      const float e = fmaf(y0, U0, fmaf(y1, U1, U2));
      const float den = fmaf(U0, U0, fmaf(U1, U1, fmaf(V0, V0, V1 * V1)));
      const float rhs = (float)maxr * den;
      const float mg = fmaf(cf[10], rhs, cf[9]);
      const float diff = fmaf(e, e, -rhs);
      const int in_ref = sampson(F, x0, x1, y0, y1) <= maxr;
      ++n;
      inl += in_ref;
      if (fabsf(diff) <= mg) {
        ++und;
      } else if ((diff < -mg) != in_ref) {
        ++bad;
        if (bad < 5) printf("BAD m=%d diff=%g mg=%g ref=%d\n", m, diff, mg, in_ref);
      }
    }
  }
  printf("maxr=%g points=%ld inliers=%ld undecided=%ld (%.4f%%) wrong=%ld\n", maxr, n, inl, und,
         100.0 * und / n, bad);
  return bad != 0;
}
