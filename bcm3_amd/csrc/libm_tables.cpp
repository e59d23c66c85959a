// libm_tables.cpp -- the data tables of the host libm's pow, for xm::pow_glibc (libm_exact.h).
//
// glibc's pow (e_pow.c since 2.28) reads two constant tables, __pow_log_data and __exp_data. They
// are not exported, so they are located in the libm this process has loaded: dl_iterate_phdr over
// its readable segments, searching for the heads of both structures (the ln2 split followed by the
// polynomial's -1/2; 128/ln2 followed by the rounding shift 1.5 * 2^52), then checked entry by
// entry (every invc of the log table in [0.7, 1.45] with a zero pad, every exp table entry within
// 2^-45 of 2^(i/128), the first one exactly 1). Nothing is copied into this repository: without a
// matching libm, bcm3_make_pow_tables computes tables of the same layout (the subinterval centres'
// reciprocals and logarithms, 2^(i/128), the Taylor coefficients), with which the same algorithm
// is accurate to about 1 ulp -- no longer glibc's bits.
#include <link.h>

#include <cmath>
#include <cstdint>
#include <cstring>

#include "libm_exact.h"

namespace {

struct Found {
    const double* logd = nullptr;
    const double* expd = nullptr;
};

constexpr uint64_t kLn2Hi = 0x3fe62e42fefa3800ull, kLn2Lo = 0x3d2ef35793c76730ull, kMinusHalf = 0xbfe0000000000000ull;
constexpr uint64_t kShift = 0x4338000000000000ull;

uint64_t bits(double x)
{
    uint64_t b;
    std::memcpy(&b, &x, 8);
    return b;
}

bool log_ok(const double* p)
{
    for (int i = 0; i < 128; i++) {
        const double* e = p + 9 + 4 * i;
        if (!(e[0] >= 0.7 && e[0] <= 1.45) || e[1] != 0.0 || !(std::fabs(e[2]) < 0.4)) return false;
    }
    return true;
}

bool exp_ok(const double* p)
{
    // invln2N, shift, negln2hiN, negln2loN, C2..C5, then exp2_shift and exp2_poly[5]: the table
    // follows 14 doubles
    const double inv = 128.0 / std::log(2.0);
    if (std::fabs(p[0] - inv) > 1e-12 * inv || bits(p[1]) != kShift) return false;
    const uint64_t* t = reinterpret_cast<const uint64_t*>(p + 14);
    if (t[0] != 0 || t[1] != 0x3ff0000000000000ull) return false;
    for (int i = 0; i < 128; i++) {
        double v;
        const uint64_t sb = t[2 * i + 1] + ((uint64_t)i << 45);
        std::memcpy(&v, &sb, 8);
        const double ref = std::exp2(i / 128.0);
        if (!(std::fabs(v - ref) <= ref * 0x1p-45)) return false;
    }
    return true;
}

int scan(struct dl_phdr_info* info, size_t, void* data)
{
    Found& f = *static_cast<Found*>(data);
    if (!info->dlpi_name || !std::strstr(info->dlpi_name, "libm.so")) return 0;
    for (int h = 0; h < info->dlpi_phnum; h++) {
        const ElfW(Phdr)& ph = info->dlpi_phdr[h];
        if (ph.p_type != PT_LOAD || !(ph.p_flags & PF_R) || (ph.p_flags & PF_W)) continue;
        const uintptr_t lo = (info->dlpi_addr + ph.p_vaddr + 7) & ~(uintptr_t)7;
        const uintptr_t hi = info->dlpi_addr + ph.p_vaddr + ph.p_filesz;
        for (uintptr_t a = lo; a + 8 * (9 + 4 * 128) <= hi || a + 8 * (14 + 256) <= hi; a += 8) {
            const uint64_t* w = reinterpret_cast<const uint64_t*>(a);
            if (!f.logd && a + 8 * (9 + 4 * 128) <= hi && w[0] == kLn2Hi && w[1] == kLn2Lo && w[2] == kMinusHalf &&
                log_ok(reinterpret_cast<const double*>(a)))
                f.logd = reinterpret_cast<const double*>(a);
            if (!f.expd && a + 8 * (14 + 256) <= hi && w[1] == kShift && exp_ok(reinterpret_cast<const double*>(a)))
                f.expd = reinterpret_cast<const double*>(a);
        }
    }
    return (f.logd && f.expd) ? 1 : 0;
}

}  // namespace

// fills *out from the loaded libm; false when either table is not found
bool bcm3_find_glibc_pow(xm::GlibcPow* out)
{
    // the process's libm (linked by this library for the host side)
    volatile double probe = std::pow(2.0, 0.5);
    (void)probe;
    Found f;
    dl_iterate_phdr(scan, &f);
    if (!f.logd || !f.expd) return false;
    std::memcpy(&out->ln2hi, f.logd, sizeof(double) * (9 + 4 * 128));
    out->invln2N = f.expd[0];
    out->shift = f.expd[1];
    out->negln2hiN = f.expd[2];
    out->negln2loN = f.expd[3];
    std::memcpy(out->C, f.expd + 4, sizeof(double) * 4);
    std::memcpy(out->exptab, f.expd + 14, sizeof(uint64_t) * 256);
    out->ok = 1;
    return true;
}

void bcm3_make_pow_tables(xm::GlibcPow* out)
{
    std::memset(out, 0, sizeof(*out));
    // ln2 = LN2_1 + LN2_2 + LN2_3 (libm_exact.h), LN2_1 with 42 significant bits: k ln2hi exact
    out->ln2hi = xm::LN2_1;
    out->ln2lo = xm::LN2_2 + xm::LN2_3;
    // log1p(r) = r - r^2/2 + ar3 (A1 + r A2 + ar2 (A3 + r A4 + ar2 (A5 + r A6))), ar = -r/2
    const double A[7] = {-0.5, -2.0 / 3.0, 0.5, 0.8, -2.0 / 3.0, -8.0 / 7.0, 1.0};
    std::memcpy(out->A, A, sizeof(A));
    // subinterval i of z in [0x3fe6955500000000, +2^52): invc near 1/centre with 8 significant
    // bits (so that z invc - 1 is exact), logc = -log(invc) rounded to a multiple of 2^-43 (so that
    // k ln2hi + logc is exact), logctail the rest
    for (int i = 0; i < 128; i++) {
        const uint64_t cb = 0x3fe6955500000000ull + ((uint64_t)i << 45) + (1ull << 44);
        double c;
        std::memcpy(&c, &cb, 8);
        const double scale = (c >= 1.0) ? 256.0 : 128.0;
        const double invc = std::nearbyint(scale / c) / scale;
        const long double lc = -logl((long double)invc);
        const double logc = std::nearbyint((double)(lc * 0x1p43L)) * 0x1p-43;
        out->logtab[i][0] = invc;
        out->logtab[i][2] = logc;
        out->logtab[i][3] = (double)(lc - (long double)logc);
    }
    out->invln2N = 128.0 / xm::LN2_1 / (1.0 + (xm::LN2_2 + xm::LN2_3) / xm::LN2_1);
    out->shift = 0x1.8p52;
    out->negln2hiN = -xm::LN2_1 / 128.0;
    out->negln2loN = -(xm::LN2_2 + xm::LN2_3) / 128.0;
    const double C[4] = {0.5, 1.0 / 6.0, 1.0 / 24.0, 1.0 / 120.0};
    std::memcpy(out->C, C, sizeof(C));
    for (int i = 0; i < 128; i++) {
        const long double v = exp2l((long double)i / 128.0L);
        const double vd = (double)v;
        const double tail = (double)((v - (long double)vd) / (long double)vd);
        out->exptab[2 * i] = bits(tail);
        out->exptab[2 * i + 1] = bits(vd) - ((uint64_t)i << 45);
    }
    out->ok = 1;
}

// the tables every device copy is filled from: the loaded libm's, else computed ones (BCM3_POW=
// computed forces those, for tests); *from_libm 1 for the former
#include <cstdlib>
#include <mutex>
const xm::GlibcPow* bcm3_pow_tables(int* from_libm)
{
    static std::once_flag once;
    static xm::GlibcPow t;
    static int found = 0;
    std::call_once(once, [] {
        const char* env = std::getenv("BCM3_POW");
        found = (!(env && !std::strcmp(env, "computed")) && bcm3_find_glibc_pow(&t)) ? 1 : 0;
        if (!found) bcm3_make_pow_tables(&t);
    });
    if (from_libm) *from_libm = found;
    return &t;
}
