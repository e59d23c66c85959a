// Accuracy of rsq-seeded Goldschmidt square roots with 2 vs 1 final corrections (ulp vs IEEE sqrt).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void k(const double* xs, double* out, int n)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double x = xs[i];
    double r = __builtin_amdgcn_rsq(x);
    double g = x * r, hh = 0.5 * r;
    double e = __builtin_fma(-g, hh, 0.5);
    g = __builtin_fma(g, e, g);
    hh = __builtin_fma(hh, e, hh);
    double d = __builtin_fma(-g, g, x);
    double g1 = __builtin_fma(d, hh, g);  // one correction
    d = __builtin_fma(-g1, g1, x);
    double g2 = __builtin_fma(d, hh, g1);  // two corrections (current fsqrt)
    out[3 * i] = g1;
    out[3 * i + 1] = g2;
    out[3 * i + 2] = sqrt(x);
}

static double ulps(double a, double b)
{
    if (a == b) return 0;
    int64_t x, y;
    std::memcpy(&x, &a, 8);
    std::memcpy(&y, &b, 8);
    return (double)llabs(x - y);
}

int main()
{
    const int n = 1 << 22;
    std::vector<double> x(n);
    uint64_t s = 999;
    for (int i = 0; i < n; i++) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        double m = 1.0 + (double)(s >> 11) / 9007199254740992.0;
        x[i] = ldexp(m, (int)((s >> 3) % 400) - 200);
    }
    double *dx, *d;
    (void)hipMalloc(&dx, n * 8);
    (void)hipMalloc(&d, 3 * n * 8);
    (void)hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(dx, d, n);
    std::vector<double> o(3 * n);
    (void)hipMemcpy(o.data(), d, 3 * n * 8, hipMemcpyDeviceToHost);
    double m1 = 0, m2 = 0;
    long c1 = 0, c2 = 0;
    for (int i = 0; i < n; i++) {
        double w = std::sqrt(x[i]);
        double u1 = ulps(o[3 * i], w), u2 = ulps(o[3 * i + 1], w);
        m1 = fmax(m1, u1);
        m2 = fmax(m2, u2);
        c1 += u1 > 0;
        c2 += u2 > 0;
    }
    printf("sqrt: 1 correction max ulp %.0f (%ld not CR); 2 corrections max ulp %.0f (%ld not CR) of %d\n", m1, c1,
           m2, c2, n);
    return 0;
}
