/*
 * flopcount.hpp -- TEST INFRASTRUCTURE (oracle). Never linked into the product.
 *
 * Op-counting build of the C restatement (F_alg "frozen in the fixture by
 * op-counting in the CPU restatement"). The oracle's C sources (popk_glue.c, ode_driver.c,
 * backend_restated.c) are compiled as C++ with this header force-included (oracle/Makefile,
 * target libflops.so): `double` becomes `fd`, a struct holding one double whose arithmetic
 * operators and math functions do the same IEEE operation and add to a thread-local counter.
 * Counting rule: +, -, *, / and fma count 1 flop each; exp, log, log1p, pow,
 * sqrt, erf count 1 each; comparisons, fabs, floor, negation, copies and conversions count 0.
 * The values are bit-identical to liboracle.so (both are built without FP contraction), which
 * tests/test_flops.py checks before trusting the count.
 */
#pragma once
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <float.h>
#include <math.h>
#include <pthread.h>
#include <xmmintrin.h>
#include <emmintrin.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

extern thread_local long long orc_flop_counter;

struct fd {
    double v;
    fd() = default;
    constexpr fd(double x) : v(x) {}
    template <class I, class = typename std::enable_if<std::is_integral<I>::value>::type>
    constexpr fd(I x) : v((double)x) {}
    explicit operator int() const { return (int)v; }
    explicit operator long() const { return (long)v; }
    explicit operator long long() const { return (long long)v; }
    explicit operator unsigned() const { return (unsigned)v; }
    explicit operator bool() const { return v != 0.0; }
    explicit operator float() const { return (float)v; }
    fd operator-() const { return fd(-v); }
    fd operator+() const { return *this; }
    fd& operator+=(fd o) { ++orc_flop_counter; v += o.v; return *this; }
    fd& operator-=(fd o) { ++orc_flop_counter; v -= o.v; return *this; }
    fd& operator*=(fd o) { ++orc_flop_counter; v *= o.v; return *this; }
    fd& operator/=(fd o) { ++orc_flop_counter; v /= o.v; return *this; }
};
static_assert(sizeof(fd) == sizeof(double), "fd must be layout-compatible with double");

inline fd operator+(fd a, fd b) { ++orc_flop_counter; return fd(a.v + b.v); }
inline fd operator-(fd a, fd b) { ++orc_flop_counter; return fd(a.v - b.v); }
inline fd operator*(fd a, fd b) { ++orc_flop_counter; return fd(a.v * b.v); }
inline fd operator/(fd a, fd b) { ++orc_flop_counter; return fd(a.v / b.v); }
inline bool operator<(fd a, fd b) { return a.v < b.v; }
inline bool operator>(fd a, fd b) { return a.v > b.v; }
inline bool operator<=(fd a, fd b) { return a.v <= b.v; }
inline bool operator>=(fd a, fd b) { return a.v >= b.v; }
inline bool operator==(fd a, fd b) { return a.v == b.v; }
inline bool operator!=(fd a, fd b) { return a.v != b.v; }
inline bool operator!(fd a) { return !a.v; }

#define FD_FN1(name)                                                        \
    inline fd name(fd a) { ++orc_flop_counter; return fd(std::name(a.v)); }
FD_FN1(exp)
FD_FN1(log)
FD_FN1(log1p)
FD_FN1(sqrt)
FD_FN1(erf)
FD_FN1(erfc)
#undef FD_FN1
inline fd pow(fd a, fd b) { ++orc_flop_counter; return fd(std::pow(a.v, b.v)); }
inline fd fma(fd a, fd b, fd c) { ++orc_flop_counter; return fd(std::fma(a.v, b.v, c.v)); }
inline fd fabs(fd a) { return fd(std::fabs(a.v)); }
inline fd floor(fd a) { return fd(std::floor(a.v)); }
inline fd fmax(fd a, fd b) { return fd(std::fmax(a.v, b.v)); }
inline fd fmin(fd a, fd b) { return fd(std::fmin(a.v, b.v)); }
inline bool isnan_fd(fd a) { return std::isnan(a.v); }
inline bool isinf_fd(fd a) { return std::isinf(a.v); }
inline bool isfinite_fd(fd a) { return std::isfinite(a.v); }

#undef isnan
#undef isinf
#undef isfinite
#define isnan(x) isnan_fd(fd(x))
#define isinf(x) isinf_fd(fd(x))
#define isfinite(x) isfinite_fd(fd(x))
#define double fd
