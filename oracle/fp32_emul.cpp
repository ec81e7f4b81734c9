/*
 * fp32_emul.cpp -- TEST INFRASTRUCTURE ONLY: the oracle's algorithm in single precision.
 *
 * The device computes in fp32; the oracle restates the reference (Bullet, fp64) in fp64.  How far
 * apart may the two be?  This build answers it with the oracle itself: pgx_oracle.c compiled
 * unchanged as C++ with every `double` replaced by a one-double struct (r32) whose arithmetic
 * operators, literals and math functions round every result to the nearest float -- the same
 * algorithm, in the same order, evaluated in fp32 arithmetic.  Its distance from the fp64 build
 * on the same inputs is the rounding envelope of the restated algorithm at the device's
 * precision (tests/test_gpu_fp32_envelope.py compares the device's deviation with it).  Like
 * flops_count.cpp the struct has the size, alignment and register class of a double, so the
 * library keeps the oracle's C ABI and oracle/oracle.py drives it like the plain build.
 *
 * Rounded: + - * / (and the compound forms), sqrt and the transcendentals (evaluated in fp64,
 * then rounded: at most one ulp of float from a correctly rounded fp32 function), every
 * conversion from a double or integer (literals and constants become floats).  Comparisons,
 * fabs / rint / ceil and unary minus are exact in either precision.
 */
#include <math.h>
#include <stdint.h>

#include <type_traits>

struct r32 {
    double v;
    static double rd(double x) { return (double)(float)x; }
    r32() = default;
    constexpr r32(double x, int) : v(x) {}
    r32(double x) : v(rd(x)) {}
    explicit operator double() const { return v; }
    explicit operator float() const { return (float)v; }
    explicit operator int() const { return (int)v; }
    explicit operator int64_t() const { return (int64_t)v; }
    explicit operator uint8_t() const { return (uint8_t)v; }
    r32 operator-() const { return r32(-v, 0); }
    r32 operator+() const { return *this; }
    r32& operator+=(r32 o) { v = rd(v + o.v); return *this; }
    r32& operator-=(r32 o) { v = rd(v - o.v); return *this; }
    r32& operator*=(r32 o) { v = rd(v * o.v); return *this; }
    r32& operator/=(r32 o) { v = rd(v / o.v); return *this; }
};
static_assert(sizeof(r32) == sizeof(double) && alignof(r32) == alignof(double), "r32 must be a double");
static_assert(std::is_trivially_copyable<r32>::value && std::is_standard_layout<r32>::value, "r32 layout");

template <class T>
using arith = typename std::enable_if<std::is_arithmetic<T>::value, int>::type;

/* a float result of two floats: the product / sum of two floats is exact in double for +, -, *
 * (24 + 24 bits), so rounding the double result once is fp32 arithmetic; / and sqrt of floats
 * rounded from double are correctly rounded as well (double has > 2 * 24 + 2 bits) */
#define R_BINOP(OP)                                                                                 \
    static inline r32 operator OP(r32 a, r32 b) { return r32(a.v OP b.v); }                          \
    template <class T, arith<T> = 0>                                                                \
    static inline r32 operator OP(r32 a, T b) { return r32(a.v OP r32::rd((double)b)); }             \
    template <class T, arith<T> = 0>                                                                \
    static inline r32 operator OP(T a, r32 b) { return r32(r32::rd((double)a) OP b.v); }
R_BINOP(+)
R_BINOP(-)
R_BINOP(*)
R_BINOP(/)
#undef R_BINOP

#define R_CMP(OP)                                                                             \
    static inline bool operator OP(r32 a, r32 b) { return a.v OP b.v; }                        \
    template <class T, arith<T> = 0>                                                          \
    static inline bool operator OP(r32 a, T b) { return a.v OP (double)b; }                    \
    template <class T, arith<T> = 0>                                                          \
    static inline bool operator OP(T a, r32 b) { return (double)a OP b.v; }
R_CMP(<)
R_CMP(<=)
R_CMP(>)
R_CMP(>=)
R_CMP(==)
R_CMP(!=)
#undef R_CMP

static inline r32 sqrt(r32 a) { return r32(::sqrt(a.v)); }
static inline r32 sin(r32 a) { return r32(::sin(a.v)); }
static inline r32 cos(r32 a) { return r32(::cos(a.v)); }
static inline r32 acos(r32 a) { return r32(::acos(a.v)); }
static inline r32 asin(r32 a) { return r32(::asin(a.v)); }
static inline r32 atan2(r32 a, r32 b) { return r32(::atan2(a.v, b.v)); }
static inline r32 cbrt(r32 a) { return r32(::cbrt(a.v)); }
static inline r32 pow(r32 a, r32 b) { return r32(::pow(a.v, b.v)); }
static inline r32 fabs(r32 a) { return r32(::fabs(a.v), 0); }
static inline r32 rint(r32 a) { return r32(::rint(a.v), 0); }
static inline r32 ceil(r32 a) { return r32(::ceil(a.v), 0); }

#define PGXO_PHASE(k) ((void)0)
#define double r32
#include "pgx_oracle.c"
#undef double
