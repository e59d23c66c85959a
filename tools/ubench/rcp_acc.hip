// Accuracy of v_rcp_f64 / v_rsq_f64 seeds and of 1 or 2 Newton steps (max ulp error vs IEEE).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

__global__ void k(const double* x, double* out, int n)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double b = x[i];
    double r = __builtin_amdgcn_rcp(b);
    double e = __builtin_fma(-b, r, 1.0);
    double r1 = __builtin_fma(e, r, r);
    e = __builtin_fma(-b, r1, 1.0);
    double r2 = __builtin_fma(e, r1, r1);
    // quotient a/b with one-step reciprocal: q = a*r1; e = fma(-b,q,a); q = fma(e,r1,q)
    double a = x[(i + 7) % n] * 3.0;
    double q1 = a * r1, eq1 = __builtin_fma(-b, q1, a);
    q1 = __builtin_fma(eq1, r1, q1);
    double q2 = a * r2, eq2 = __builtin_fma(-b, q2, a);
    q2 = __builtin_fma(eq2, r2, q2);
    out[6 * i + 0] = r;
    out[6 * i + 1] = r1;
    out[6 * i + 2] = r2;
    out[6 * i + 3] = q1;
    out[6 * i + 4] = q2;
    out[6 * i + 5] = a / b;
}

static double ulps(double got, double want)
{
    if (got == want) return 0.0;
    int64_t a, b;
    std::memcpy(&a, &got, 8);
    std::memcpy(&b, &want, 8);
    return (double)llabs(a - b);
}

int main()
{
    const int n = 1 << 22;
    std::vector<double> x(n);
    uint64_t s = 12345;
    for (int i = 0; i < n; i++) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        double m = 1.0 + (double)(s >> 11) / 9007199254740992.0;
        int ex = (int)((s >> 3) % 200) - 100;
        x[i] = ldexp(m, ex) * ((s & 1) ? 1 : -1);
    }
    double *dx, *dout;
    hipMalloc(&dx, n * 8);
    hipMalloc(&dout, 6 * n * 8);
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(dx, dout, n);
    std::vector<double> o(6 * n);
    hipMemcpy(o.data(), dout, 6 * n * 8, hipMemcpyDeviceToHost);
    double m0 = 0, m1 = 0, m2 = 0, mq1 = 0, mq2 = 0;
    long nq1 = 0, nq2 = 0;
    for (int i = 0; i < n; i++) {
        double want = 1.0 / x[i];
        m0 = fmax(m0, ulps(o[6 * i], want));
        m1 = fmax(m1, ulps(o[6 * i + 1], want));
        m2 = fmax(m2, ulps(o[6 * i + 2], want));
        double u1 = ulps(o[6 * i + 3], o[6 * i + 5]), u2 = ulps(o[6 * i + 4], o[6 * i + 5]);
        mq1 = fmax(mq1, u1);
        mq2 = fmax(mq2, u2);
        nq1 += u1 > 0;
        nq2 += u2 > 0;
    }
    printf("rcp seed max ulp %.0f; 1 Newton %.0f; 2 Newton %.0f\n", m0, m1, m2);
    printf("quotient with 1-step rcp: max ulp %.0f (%ld of %d not correctly rounded); 2-step: max ulp %.0f (%ld)\n",
           mq1, nq1, n, mq2, nq2);
    return 0;
}
