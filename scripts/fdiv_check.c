/* CPU proof-by-testing of the reciprocal-form division and the fix-up square root used by the Adam
 * epilogues (rc_common.h rc_div_bc2s / rc_div_recip / rc_sqrt_rn) against IEEE float32 x / y and
 * sqrtf (glibc, correctly rounded), with fmaf as the hardware's fused multiply-add.
 *
 *   gcc -O2 -o /tmp/fdiv_check scripts/fdiv_check.c -lm && /tmp/fdiv_check
 *
 * 1. q = x * r; q += (x - q * y) * r (both fma) with r = RN(1 / y): every mantissa of y (exponent 0)
 *    against 40 x each, then 3e8 random (x, y) over all exponents, counted where x, q and y lie in
 *    [2^-100, 2^100] (the rc_div_recip condition; rc_div_bc2s's operands always do).
 * 2. s = sqrt_approx(v) (the correctly rounded root perturbed by -1 / 0 / +1 ulp: v_sqrt_f32 is within
 *    1 ulp), then the neighbour fix-up, for v in [2^-97, 2^127): 3e8 random v.
 * Expected output: 0 bad in every line. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static float bits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t ub(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float divr(float x, float y, float r) { float q = x * r; float e = fmaf(-y, q, x); return fmaf(e, r, q); }
static float sqrt_fix(float v, int pert) {
  float s = sqrtf(v); s = bits(ub(s) + pert);
  float sm = bits(ub(s) - 1), sp = bits(ub(s) + 1);
  float t = (fmaf(-sm, s, v) <= 0.f) ? sm : s;
  return (fmaf(-sp, s, v) > 0.f) ? sp : t;
}
static uint64_t rs = 88172645463325252ull;
static uint64_t rnd(void) { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return rs; }
int main(void) {
  long bad = 0, n = 0;
  for (uint32_t my = 0; my < (1u << 23); my++) {
    float y = bits((127u << 23) | my), r = 1.0f / y;
    for (int k = 0; k < 40; k++) {
      uint32_t mx = k == 0 ? 0 : (k == 1 ? 0x7fffff : (k == 2 ? my : (k == 3 ? (my + 1) & 0x7fffff : (k == 4 ? (my - 1) & 0x7fffff : (rnd() & 0x7fffff)))));
      float x = bits(((127u + (k & 1)) << 23) | mx);
      n++;
      if (ub(divr(x, y, r)) != ub(x / y)) bad++;
    }
  }
  printf("division, every mantissa of y: %ld bad / %ld\n", bad, n);
  bad = n = 0;
  for (long i = 0; i < 300000000L; i++) {
    float y = bits(((uint32_t)(1 + rnd() % 253) << 23) | (rnd() & 0x7fffff)), r = 1.0f / y;
    float x = bits(((rnd() & 1) << 31) | ((uint32_t)(1 + rnd() % 253) << 23) | (rnd() & 0x7fffff));
    float q = divr(x, y, r), ax = fabsf(x), aq = fabsf(q), ay = fabsf(y);
    if (!(ax >= 0x1p-100f && ax <= 0x1p100f && aq >= 0x1p-100f && aq <= 0x1p100f && ay >= 0x1p-100f && ay <= 0x1p100f)) continue;
    n++;
    if (ub(q) != ub(x / y)) bad++;
  }
  printf("division, random in range: %ld bad / %ld\n", bad, n);
  bad = n = 0;
  for (long i = 0; i < 300000000L; i++) {
    float v = bits(((uint32_t)(30 + rnd() % 224) << 23) | (rnd() & 0x7fffff));
    int pert = (int)(rnd() % 3) - 1;
    n++;
    if (ub(sqrt_fix(v, pert)) != ub(sqrtf(v))) bad++;
  }
  printf("square root, v in [2^-97, 2^127): %ld bad / %ld\n", bad, n);
  return 0;
}
