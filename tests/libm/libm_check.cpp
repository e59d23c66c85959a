// Host check of bcm3_amd/csrc/libm_exact.h (the device code, compiled for the host) against the
// host's glibc and against quad precision (libquadmath) as the correctly rounded truth.
//   libm_check <fn> <n> <seed>   prints: n  agree_glibc  agree_cr  glibc_cr
#include <quadmath.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "../../bcm3_amd/csrc/libm_exact.h"

bool bcm3_find_glibc_pow(xm::GlibcPow* out);  // bcm3_amd/csrc/libm_tables.cpp
void bcm3_make_pow_tables(xm::GlibcPow* out);

static double cr(__float128 v) { return (double)v; }  // quad -> double rounds to nearest

int main(int argc, char** argv)
{
    const char* fn = argv[1];
    const long n = atol(argv[2]);
    std::mt19937_64 rng(atol(argv[3]));
    std::uniform_real_distribution<double> U(0.0, 1.0);
    long ag = 0, ac = 0, gc = 0;
    static xm::GlibcPow D;
    if ((!strcmp(fn, "powglibc") || !strcmp(fn, "expglibc") || !strcmp(fn, "powhybrid")) && !bcm3_find_glibc_pow(&D)) {
        printf("tables not found\n");
        return 2;
    }
    if (!strcmp(fn, "powcomputed")) bcm3_make_pow_tables(&D);
    for (long i = 0; i < n; i++) {
        double x, mine, lib;
        __float128 q;
        if (!strcmp(fn, "exp")) {
            x = -40.0 + 80.0 * U(rng);
            mine = xm::exp(x);
            lib = exp(x);
            q = expq((__float128)x);
        } else if (!strcmp(fn, "log")) {
            x = exp(-60.0 + 120.0 * U(rng));
            mine = xm::log(x);
            lib = log(x);
            q = logq((__float128)x);
        } else if (!strcmp(fn, "log1p")) {
            x = (i % 3 == 0) ? -0.3 + 0.8 * U(rng) : exp(-40.0 + 45.0 * U(rng));
            mine = xm::log1p(x);
            lib = log1p(x);
            q = log1pq((__float128)x);
        } else if (!strcmp(fn, "erf") || !strcmp(fn, "erfc")) {
            x = (i % 2 ? -1.0 : 1.0) * ((i % 5 == 0) ? 7.0 * U(rng) : exp(-12.0 + 14.0 * U(rng)));
            const bool e = !strcmp(fn, "erf");
            mine = e ? xm::erf(x) : xm::erfc(x);
            lib = e ? erf(x) : erfc(x);
            q = e ? erfq((__float128)x) : erfcq((__float128)x);
        } else if (!strcmp(fn, "expglibc")) {
            // the range of glibc exp's main path, 2^-54 <= |x| < 512
            x = (i % 2 ? -1.0 : 1.0) * ((i % 5 == 0) ? 0x1p-54 * exp(36.0 * U(rng)) : 500.0 * U(rng) + 0x1p-50);
            mine = xm::exp_glibc(x, D);
            lib = exp(x);
            q = expq((__float128)x);
        } else if (!strcmp(fn, "powhybrid")) {
            // the device's step-size root (bdf_lane.h pow_root): the checked correctly rounded root,
            // glibc's algorithm near rounding midpoints
            const int k = 2 + (int)(i % 6);
            x = (i % 7 == 0) ? 1.0 + (U(rng) - 0.5) * 0x1p-40 : exp(-69.0 + 138.0 * U(rng));
            const double y = xm::inv_k(k);
            bool safe;
            mine = xm::pow_inv_k_checked(x, k, safe);
            if (!safe) mine = xm::pow_glibc(x, y, D);
            lib = pow(x, y);
            q = powq((__float128)x, (__float128)y);
        } else if (!strcmp(fn, "powglibc") || !strcmp(fn, "powcomputed")) {
            // the solvers' step-size roots: x in (1e-30, 1e30), some within 2^-40 of 1
            const int k = 2 + (int)(i % 6);
            x = (i % 7 == 0) ? 1.0 + (U(rng) - 0.5) * 0x1p-40 : exp(-69.0 + 138.0 * U(rng));
            const double y = xm::inv_k(k);
            mine = xm::pow_glibc(x, y, D);
            lib = pow(x, y);
            q = powq((__float128)x, (__float128)y);
        } else {
            const int k = 2 + (int)(i % 6);
            x = exp(-60.0 + 60.0 * U(rng));
            mine = xm::pow_inv_k(x, k);
            const double y = 1.0 / k;
            lib = pow(x, y);
            q = powq((__float128)x, (__float128)y);
        }
        const double c = cr(q);
        ag += (mine == lib);
        ac += (mine == c);
        gc += (lib == c);
        if (mine != c && argc > 4) printf("x=%a mine=%a cr=%a lib=%a\n", x, mine, c, lib);
    }
    printf("%ld %ld %ld %ld\n", n, ag, ac, gc);
    return 0;
}
