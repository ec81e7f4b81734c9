/*
 * flops_count.cpp -- TEST INFRASTRUCTURE ONLY: an operation-counting build of the fp64 oracle.
 *
 * The algorithmic FLOP count per env-step that SURVEY.md §8d asks for ("to be op-counted in
 * the CPU restatement and frozen as a fixture constant") is taken here: pgx_oracle.c is compiled
 * unchanged as C++ with every `double` replaced by a one-double struct (fcd) whose arithmetic
 * operators and math functions increment global counters.  The struct has the size, alignment
 * and register class of a double, so the library keeps the oracle's C ABI (pgx_config's double
 * fields, double* arrays, double returns) and oracle/oracle.py drives it like the plain build.
 *
 * Counted (fp64 operations on run-time values; constant folding of literals is not counted):
 *   add   + and - (binary), += and -=          mul   *, *=
 *   div   /, /=                                 sqrt  sqrt
 *   trans sin cos acos asin atan2 cbrt pow      cmp   < <= > >= == != (not FLOPs, reported apart)
 * rint / ceil / fabs / unary minus are not counted (rounding, sign and exponent bit operations).
 * FLOPs = add + mul + div + sqrt + trans, each 1 (an FMA would be 2; the oracle has none:
 * it is built with -ffp-contract=off).  Counters are kept per phase of the step (the
 * PGXO_PHASE marks in pgx_oracle.c: action + IK, detection, dynamics, row setup, PGS sweeps,
 * integration, observation / reward, reset, ReachAO collision check).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <type_traits>

#define PGXO_NPHASE 9   /* the phase marks of pgx_oracle.c (PGXO_PHASE) */

extern "C" {
typedef struct pgxo_flops_t {
    int64_t add, mul, div, sqrt, trans, cmp;
} pgxo_flops_t;
static pgxo_flops_t g_flops[PGXO_NPHASE];
static int g_phase;
/* counters per phase [PGXO_NPHASE]; clear resets them */
void pgxo_flops_read(pgxo_flops_t* out, int clear) {
    memcpy(out, g_flops, sizeof g_flops);
    if (clear) memset(g_flops, 0, sizeof g_flops);
}
int pgxo_flops_nphase(void) { return PGXO_NPHASE; }
}
#define pgxo_flops g_flops[g_phase]
#define PGXO_PHASE(k) (g_phase = (k))
/* model constants computed per call (the contact breaking thresholds): not counted */
#define PGXO_CONST_BEGIN pgxo_flops_t pgxo_saved_[PGXO_NPHASE]; memcpy(pgxo_saved_, g_flops, sizeof g_flops)
#define PGXO_CONST_END memcpy(g_flops, pgxo_saved_, sizeof g_flops)

struct fcd {
    double v;
    fcd() = default;
    constexpr fcd(double x) : v(x) {}
    explicit operator double() const { return v; }
    explicit operator float() const { return (float)v; }
    explicit operator int() const { return (int)v; }
    explicit operator int64_t() const { return (int64_t)v; }
    explicit operator uint8_t() const { return (uint8_t)v; }
    fcd operator-() const { return fcd(-v); }
    fcd operator+() const { return *this; }
    fcd& operator+=(fcd o) { pgxo_flops.add++; v += o.v; return *this; }
    fcd& operator-=(fcd o) { pgxo_flops.add++; v -= o.v; return *this; }
    fcd& operator*=(fcd o) { pgxo_flops.mul++; v *= o.v; return *this; }
    fcd& operator/=(fcd o) { pgxo_flops.div++; v /= o.v; return *this; }
};
static_assert(sizeof(fcd) == sizeof(double) && alignof(fcd) == alignof(double), "fcd must be a double");
static_assert(std::is_trivially_copyable<fcd>::value && std::is_standard_layout<fcd>::value, "fcd layout");

template <class T>
using arith = typename std::enable_if<std::is_arithmetic<T>::value, int>::type;

#define CD_BINOP(OP, CNT)                                                                   \
    static inline fcd operator OP(fcd a, fcd b) { pgxo_flops.CNT++; return fcd(a.v OP b.v); }    \
    template <class T, arith<T> = 0>                                                        \
    static inline fcd operator OP(fcd a, T b) { pgxo_flops.CNT++; return fcd(a.v OP (double)b); } \
    template <class T, arith<T> = 0>                                                        \
    static inline fcd operator OP(T a, fcd b) { pgxo_flops.CNT++; return fcd((double)a OP b.v); }
CD_BINOP(+, add)
CD_BINOP(-, add)
CD_BINOP(*, mul)
CD_BINOP(/, div)
#undef CD_BINOP

#define CD_CMP(OP)                                                                            \
    static inline bool operator OP(fcd a, fcd b) { pgxo_flops.cmp++; return a.v OP b.v; }       \
    template <class T, arith<T> = 0>                                                          \
    static inline bool operator OP(fcd a, T b) { pgxo_flops.cmp++; return a.v OP (double)b; }  \
    template <class T, arith<T> = 0>                                                          \
    static inline bool operator OP(T a, fcd b) { pgxo_flops.cmp++; return (double)a OP b.v; }
CD_CMP(<)
CD_CMP(<=)
CD_CMP(>)
CD_CMP(>=)
CD_CMP(==)
CD_CMP(!=)
#undef CD_CMP

static inline fcd sqrt(fcd a) { pgxo_flops.sqrt++; return fcd(::sqrt(a.v)); }
static inline fcd sin(fcd a) { pgxo_flops.trans++; return fcd(::sin(a.v)); }
static inline fcd cos(fcd a) { pgxo_flops.trans++; return fcd(::cos(a.v)); }
static inline fcd acos(fcd a) { pgxo_flops.trans++; return fcd(::acos(a.v)); }
static inline fcd asin(fcd a) { pgxo_flops.trans++; return fcd(::asin(a.v)); }
static inline fcd atan2(fcd a, fcd b) { pgxo_flops.trans++; return fcd(::atan2(a.v, b.v)); }
static inline fcd cbrt(fcd a) { pgxo_flops.trans++; return fcd(::cbrt(a.v)); }
static inline fcd pow(fcd a, fcd b) { pgxo_flops.trans++; return fcd(::pow(a.v, b.v)); }
static inline fcd fabs(fcd a) { return fcd(::fabs(a.v)); }
static inline fcd rint(fcd a) { return fcd(::rint(a.v)); }
static inline fcd ceil(fcd a) { return fcd(::ceil(a.v)); }

#define double fcd
#include "pgx_oracle.c"
#undef double
#undef pgxo_flops
