/* div_rn's identity (mc_bp_kernels.inl): for rb = RN(1 / b), RN(RN(a rb) + (a - b RN(a rb)) rb), the
 * remainder exact by FMA, equals the IEEE quotient a / b (Markstein).  Checked on operands of S1's
 * per-pixel divisions (the unprojection (u - cx) z / fx, the voxel index (p - vmin) / vs, quotients
 * within a few ulps of integers where floor() is decided) and on random doubles of many exponents.
 *   div_check <samples>   ->  prints "n=<samples> bad=<mismatches>"                              */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s = 88172645463325252ull;
static uint64_t xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double u01(void) { return (double)(xr() >> 11) * (1.0 / 9007199254740992.0); }

int main(int argc, char **argv)
{
    const long n = argc > 1 ? atol(argv[1]) : 10000000;
    const double vs[] = {0.01, 0.0404, 0.04, 0.02, 0.005};
    long bad = 0;
    for (long i = 0; i < n; i++) {
        double a, b;
        switch (i % 5) {
        case 0: a = (u01() * 2 - 1) * 5000.0 * u01(); b = 100.0 + 2000.0 * u01(); break;  /* (u - cx) z / fx */
        case 1: a = u01() * 20.0; b = vs[xr() % 5]; break;                                  /* (p - vmin) / vs */
        case 2: {                                                                           /* near k b */
            b = (xr() & 1) ? vs[xr() % 5] : 100.0 + 2000.0 * u01();
            a = (double)(xr() % 4096) * b;
            for (int d = (int)(xr() % 7) - 3; d != 0; d += d > 0 ? -1 : 1) a = nextafter(a, d > 0 ? INFINITY : -INFINITY);
            break;
        }
        default: {                                                                          /* exponents 2^-255..2^256 */
            uint64_t x = (xr() & 0x001FFFFFFFFFFFFFull) | ((uint64_t)(768 + xr() % 512) << 52);
            uint64_t y = (xr() & 0x001FFFFFFFFFFFFFull) | ((uint64_t)(768 + xr() % 512) << 52);
            memcpy(&a, &x, 8);
            memcpy(&b, &y, 8);
            if (xr() & 1) a = -a;
        }
        }
        const double rb = 1.0 / b, q0 = a * rb, r = fma(-b, q0, a), q1 = fma(r, rb, q0), q = a / b;
        if (memcmp(&q, &q1, 8) != 0) {
            if (bad < 5) printf("mismatch a=%.17g b=%.17g q=%.17g q1=%.17g\n", a, b, q, q1);
            bad++;
        }
    }
    printf("n=%ld bad=%ld\n", n, bad);
    return bad != 0;
}
