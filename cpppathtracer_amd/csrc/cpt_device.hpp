// cpt_device.hpp — device-side building blocks of the integrator (gfx950).
//
// Every function here restates a piece of the reference hot path with the reference's
// floating-point semantics (file:line cited per function).  Compiled with
// -ffp-contract=off and IEEE f32/f64 division and sqrt, so each expression rounds exactly as
// written; transcendentals use the deterministic double-precision sequences defined in
// DESIGN.md §Numerics (same sequences as the CPU oracle), so GPU and oracle agree bit for bit.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cpt_fm_tables.hpp"

namespace cpt {

// ------------------------------------------------------------------------------------
// float3 with the vendored helper_math.h semantics (Common/helper_math.h).
// ------------------------------------------------------------------------------------
struct v3 { float x, y, z; };

__device__ __forceinline__ v3 mk(float x, float y, float z) { return v3{x, y, z}; }
__device__ __forceinline__ v3 mk1(float s) { return v3{s, s, s}; }
__device__ __forceinline__ v3 operator+(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ v3 operator-(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ v3 operator*(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ v3 operator*(float s, v3 a) { return mk(s * a.x, s * a.y, s * a.z); }   // :834-837
__device__ __forceinline__ v3 operator*(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ v3 operator/(v3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }   // :1013-1016
__device__ __forceinline__ v3 operator-(v3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }  // :1264-1267
// 1.0f / x, correctly rounded, in 3 ops instead of the ~10-op IEEE divide sequence: v_rcp_f32
// and one Newton step (fma) give the IEEE reciprocal of every float with 2^-126 <= |x| <
// 2^126 (checked for all 2^32 patterns, tools/exact_rcp_check.hip, test_rcp_exhaustive); +-0
// and +-inf take v_rcp_f32's own +-inf / +-0 (the step makes a NaN there).  Callers pass only
// such x: sqrtf outputs (never subnormal, never >= 2^64) and unit-vector components >= 1e-30.
__device__ __forceinline__ float rcp_f(float x) {
    const float r0 = __builtin_amdgcn_rcpf(x);
    const float r = __builtin_fmaf(__builtin_fmaf(-x, r0, 1.0f), r0, r0);
    return r == r ? r : r0;
}

__device__ __forceinline__ v3 normalize(v3 v) {                                                  // :1325-1329
    float inv = rcp_f(__builtin_sqrtf(dot(v, v)));   // host-path rsqrtf = 1/sqrtf (:78-81)
    return v * inv;
}

// sqrtf(x), correctly rounded, for x = +-0, |x| >= 2^-96, inf or NaN: the compiler's own IEEE
// sequence (v_sqrt_f32, then the candidate +-1 ulp chosen by the signs of the two fma
// residuals) without the steps that serve only |x| < 2^-96 (the 2^32 pre-scale and 2^-16
// post-scale) and +-0 / +inf (the final class select: the residual steps already return
// v_sqrt_f32's +-0 / +inf unchanged); checked for every pattern of that domain on the device
// (test_sqrt_nn_exhaustive).  Callers pass 0 or quantities far from 2^-96: 1 - z*z of floats
// z <= 1 (0, >= 2^-24, or <= -2^-24), squared lengths of near-unit vectors.
__device__ __forceinline__ float sqrt_nn_raw(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __int_as_float(__float_as_int(s) - 1), sp = __int_as_float(__float_as_int(s) + 1);
    const float rm = __builtin_fmaf(-sm, s, x), rp = __builtin_fmaf(-sp, s, x);
    const float r = rm <= 0.0f ? sm : s;
    return rp > 0.0f ? sp : r;
}
__device__ __forceinline__ float sqrt_nn(float x) { return sqrt_nn_raw(x); }
// normalize() of a vector whose squared length is 0 or >= 2^-96 (a unit vector up to rounding)
__device__ __forceinline__ v3 normalize_u(v3 v) {
    float inv = rcp_f(sqrt_nn(dot(v, v)));
    return v * inv;
}
__device__ __forceinline__ v3 cross(v3 a, v3 b) {                                               // :1436-1439
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ v3 reflect(v3 i, v3 n) { return i - (2.0f * n) * dot(n, i); }        // :1427-1430

// MIN / MAX / ABS ternary macros (ray_tracing_math.hpp:15-26)
__device__ __forceinline__ float tmin_(float a, float b) { return a < b ? a : b; }
__device__ __forceinline__ float tmax_(float a, float b) { return a > b ? a : b; }

constexpr float DEFAULT_RAY_TMAX = 1e30f;   // ray_tracing_common.h:11
constexpr float BOUNCE_RAY_TMIN = 2e-5f;    // ray_tracing_common.h:12
constexpr uint32_t MAX_RECURSION_DEPTH_SET = 32;  // path_tracer.h:13
constexpr double REF_PI = 3.14159265358979323846;

// ------------------------------------------------------------------------------------
// Deterministic transcendentals.  Double-precision sequences with
// explicit constants and explicit fused multiply-adds (no other contraction).  Identical
// sequences live in the CPU oracle (std::fma).
// ------------------------------------------------------------------------------------
namespace dm {

constexpr double LN2_HI = 6.93147180369123816490e-01;
constexpr double LN2_LO = 1.90821492927058770002e-10;
constexpr double INV_LN2 = 1.44269504088896338700e+00;
constexpr double SQRT2 = 1.41421356237309514547e+00;
constexpr double PIO2_1 = 1.57079632673412561417e+00;
constexpr double PIO2_2 = 6.07710050650619224932e-11;
constexpr double PIO2_3 = 2.02226624879595063154e-21;
constexpr double TWO_OVER_PI = 6.36619772367581382433e-01;
constexpr double PI_2_D = 1.57079632679489655800e+00;

// A double constant materialised in SGPRs where it is used (the empty asm hides its value), so
// the compiler cannot hoist the polynomials' constants out of the persistent loop into VGPRs.
__device__ __forceinline__ double kc(double c) {
    asm volatile("" : "+s"(c));
    return c;
}

__device__ __forceinline__ uint64_t dbits(double x) { return (uint64_t)__double_as_longlong(x); }
__device__ __forceinline__ double bitsd(uint64_t u) { return __longlong_as_double((long long)u); }

__device__ inline double log_pos(double x) {
    // x > 0, finite (callers handle the special cases)
    uint64_t u = dbits(x);
    int e = (int)((u >> 52) & 0x7ff);
    if (e == 0) {
        x = x * 18014398509481984.0;
        u = dbits(x);
        e = (int)((u >> 52) & 0x7ff) - 54;
    }
    e -= 1023;
    double m = bitsd((u & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL);
    if (m > SQRT2) { m = m * 0.5; e += 1; }
    double f = m - 1.0;
    double s = f / (2.0 + f);
    double s2 = s * s;
    double p = 1.0 / 25.0;
    p = __builtin_fma(s2, p, kc(1.0 / 23.0));
    p = __builtin_fma(s2, p, kc(1.0 / 21.0));
    p = __builtin_fma(s2, p, kc(1.0 / 19.0));
    p = __builtin_fma(s2, p, kc(1.0 / 17.0));
    p = __builtin_fma(s2, p, kc(1.0 / 15.0));
    p = __builtin_fma(s2, p, kc(1.0 / 13.0));
    p = __builtin_fma(s2, p, kc(1.0 / 11.0));
    p = __builtin_fma(s2, p, kc(1.0 / 9.0));
    p = __builtin_fma(s2, p, kc(1.0 / 7.0));
    p = __builtin_fma(s2, p, kc(1.0 / 5.0));
    p = __builtin_fma(s2, p, kc(1.0 / 3.0));
    double r = __builtin_fma(2.0 * s, s2 * p, 2.0 * s);
    double de = (double)e;
    return __builtin_fma(de, kc(LN2_HI), __builtin_fma(de, kc(LN2_LO), r));
}

__device__ inline double log(double x) {
    if (!(x > 0.0)) return x == 0.0 ? -__builtin_inf() : __builtin_nan("");
    if (x == __builtin_inf()) return x;
    return log_pos(x);
}

__device__ __forceinline__ double ldexp_(double x, int k) {
    if (k > 1023) { x = x * bitsd(0x7fe0000000000000ULL); k -= 1023; if (k > 1023) k = 1023; }
    if (k < -1022) { x = x * bitsd(0x0010000000000000ULL); k += 1022; if (k < -1022) k = -1022; }
    return x * bitsd((uint64_t)(k + 1023) << 52);
}

__device__ inline double exp(double x) {
    if (x != x) return x;
    if (x > 709.782712893384) return __builtin_inf();
    if (x < -745.1332191019412) return 0.0;
    double k = __builtin_floor(__builtin_fma(x, kc(INV_LN2), 0.5));
    double r = __builtin_fma(-k, kc(LN2_LO), __builtin_fma(-k, kc(LN2_HI), x));
    double p = 1.0 / 6227020800.0;
    p = __builtin_fma(r, p, kc(1.0 / 479001600.0));
    p = __builtin_fma(r, p, kc(1.0 / 39916800.0));
    p = __builtin_fma(r, p, kc(1.0 / 3628800.0));
    p = __builtin_fma(r, p, kc(1.0 / 362880.0));
    p = __builtin_fma(r, p, kc(1.0 / 40320.0));
    p = __builtin_fma(r, p, kc(1.0 / 5040.0));
    p = __builtin_fma(r, p, kc(1.0 / 720.0));
    p = __builtin_fma(r, p, kc(1.0 / 120.0));
    p = __builtin_fma(r, p, kc(1.0 / 24.0));
    p = __builtin_fma(r, p, kc(1.0 / 6.0));
    p = __builtin_fma(r, p, kc(0.5));
    p = __builtin_fma(r, p, kc(1.0));
    p = __builtin_fma(r, p, kc(1.0));
    return ldexp_(p, (int)k);
}

__device__ inline double pow(double x, double y) {
    if (y == 0.0) return 1.0;
    if (x == 1.0) return 1.0;
    if (x != x || y != y) return __builtin_nan("");
    if (x == 0.0) return y > 0.0 ? 0.0 : __builtin_inf();
    if (x < 0.0) {
        double yi = __builtin_floor(y);
        if (yi != y) return __builtin_nan("");
        double m = exp(y * log(-x));
        double half = y * 0.5;
        return (__builtin_floor(half) != half) ? -m : m;
    }
    if (x == __builtin_inf()) return y > 0.0 ? __builtin_inf() : 0.0;
    return exp(y * log_pos(x));
}

__device__ __forceinline__ float powf_(float x, float y) { return (float)pow((double)x, (double)y); }

// pow(x, 5) of schlick (ray_tracing_math.hpp:68, the integer exponent): x^2 is exact in double,
// then two rounded products -- a few ulps of double from the exact power, like pow's exp(5 log x),
// at a fraction of its cost.  The oracle's dm_pow5f is the same three products.
__device__ __forceinline__ float pow5f(float xf) {
    const double x = (double)xf;
    const double x2 = x * x;
    return (float)(x2 * x2 * x);
}

__device__ inline double sin_poly(double r) {
    double r2 = r * r;
    double p = -1.0 / 121645100408832000.0;
    p = __builtin_fma(r2, p, kc(1.0 / 355687428096000.0));
    p = __builtin_fma(r2, p, kc(-1.0 / 1307674368000.0));
    p = __builtin_fma(r2, p, kc(1.0 / 6227020800.0));
    p = __builtin_fma(r2, p, kc(-1.0 / 39916800.0));
    p = __builtin_fma(r2, p, kc(1.0 / 362880.0));
    p = __builtin_fma(r2, p, kc(-1.0 / 5040.0));
    p = __builtin_fma(r2, p, kc(1.0 / 120.0));
    p = __builtin_fma(r2, p, kc(-1.0 / 6.0));
    return __builtin_fma(r, r2 * p, r);
}

__device__ inline double cos_poly(double r) {
    double r2 = r * r;
    double p = 1.0 / 2432902008176640000.0;
    p = __builtin_fma(r2, p, kc(-1.0 / 6402373705728000.0));
    p = __builtin_fma(r2, p, kc(1.0 / 20922789888000.0));
    p = __builtin_fma(r2, p, kc(-1.0 / 87178291200.0));
    p = __builtin_fma(r2, p, kc(1.0 / 479001600.0));
    p = __builtin_fma(r2, p, kc(-1.0 / 3628800.0));
    p = __builtin_fma(r2, p, kc(1.0 / 40320.0));
    p = __builtin_fma(r2, p, kc(-1.0 / 720.0));
    p = __builtin_fma(r2, p, kc(1.0 / 24.0));
    p = __builtin_fma(r2, p, kc(-0.5));
    return __builtin_fma(r2, p, 1.0);
}

__device__ __forceinline__ double reduce(double x, int* q) {
    double k = __builtin_floor(__builtin_fma(x, kc(TWO_OVER_PI), 0.5));
    double r = __builtin_fma(-k, kc(PIO2_3), __builtin_fma(-k, kc(PIO2_2), __builtin_fma(-k, kc(PIO2_1), x)));
    double km = k - 4.0 * __builtin_floor(k * 0.25);
    *q = (int)km;
    return r;
}

// sinf and cosf of the same argument (the BSDF lobes always need both).
__device__ inline void sincosf_(float xf, float* s_out, float* c_out) {
    double x = (double)xf;
    if (x != x || x == __builtin_inf() || x == -__builtin_inf()) {
        *s_out = __builtin_nanf("");
        *c_out = __builtin_nanf("");
        return;
    }
    int q;
    double r = reduce(x, &q);
    double sp = sin_poly(r), cp = cos_poly(r);
    double s, c;
    switch (q) {
        case 0: s = sp; c = cp; break;
        case 1: s = cp; c = -sp; break;
        case 2: s = -sp; c = -cp; break;
        default: s = -cp; c = sp; break;
    }
    *s_out = (float)s;
    *c_out = (float)c;
}

// fdlibm s_atan.c constants (public domain): atan(0.5), atan(1), atan(1.5), atan(inf) as
// hi + lo, and the minimax coefficients of atan(x) ~ x - x (aT0 z + aT1 z^2 + ...), z = x^2.
constexpr double ATAN_HI0 = 4.63647609000806093515e-01, ATAN_LO0 = 2.26987774529616870924e-17;
constexpr double ATAN_HI1 = 7.85398163397448278999e-01, ATAN_LO1 = 3.06161699786838301793e-17;
constexpr double ATAN_HI2 = 9.82793723247329054082e-01, ATAN_LO2 = 1.39033110312309984516e-17;
constexpr double ATAN_HI3 = 1.57079632679489655800e+00, ATAN_LO3 = 6.12323399573676603587e-17;
constexpr double AT0 = 3.33333333333329318027e-01, AT1 = -1.99999999998764832476e-01;
constexpr double AT2 = 1.42857142725034663711e-01, AT3 = -1.11111104054623557880e-01;
constexpr double AT4 = 9.09088713343650656196e-02, AT5 = -7.69187620504482999495e-02;
constexpr double AT6 = 6.66107313738753120669e-02, AT7 = -5.83357013379057348645e-02;
constexpr double AT8 = 4.97687799461593236017e-02, AT9 = -3.65315727442169155270e-02;
constexpr double AT10 = 1.62858201153657823623e-02;

__device__ inline double atan(double t) {
    // fdlibm's reduction to |x| < 7/16 around atan(0.5), atan(1), atan(1.5), atan(inf), with
    // one division chosen by selects, and its odd/even split of an 11-term minimax polynomial
    // (DESIGN.md §Numerics).  Identical operation sequence in the oracle (dm_atan).
    if (t != t || t == 0.0) return t;
    const double sgn = t < 0.0 ? -1.0 : 1.0;
    const double a = t < 0.0 ? -t : t;
    if (a == __builtin_inf()) return sgn * PI_2_D;
    const bool r0 = a < 0.4375, r1 = a < 0.6875, r2 = a < 1.1875, r3 = a < 2.4375;
    const double num = r0 ? a : r1 ? 2.0 * a - 1.0 : r2 ? a - 1.0 : r3 ? a - 1.5 : -1.0;
    const double den = r0 ? 1.0 : r1 ? 2.0 + a : r2 ? a + 1.0 : r3 ? 1.0 + 1.5 * a : a;
    const double hi = r1 ? ATAN_HI0 : r2 ? ATAN_HI1 : r3 ? ATAN_HI2 : ATAN_HI3;
    const double lo = r1 ? ATAN_LO0 : r2 ? ATAN_LO1 : r3 ? ATAN_LO2 : ATAN_LO3;
    const double x = num / den;
    const double z = x * x, w = z * z;
    const double s1 = z * __builtin_fma(w, __builtin_fma(w, __builtin_fma(w, __builtin_fma(w, __builtin_fma(w, kc(AT10), kc(AT8)), kc(AT6)), kc(AT4)), kc(AT2)), kc(AT0));
    const double s2 = w * __builtin_fma(w, __builtin_fma(w, __builtin_fma(w, __builtin_fma(w, kc(AT9), kc(AT7)), kc(AT5)), kc(AT3)), kc(AT1));
    const double r = r0 ? __builtin_fma(-x, s1 + s2, x) : hi - (__builtin_fma(x, s1 + s2, -lo) - x);
    return sgn * r;
}

__device__ __forceinline__ float atanf_(float x) { return (float)atan((double)x); }

__device__ inline float asinf_(float xf) {
    double x = (double)xf;
    if (x != x) return __builtin_nanf("");
    if (x > 1.0 || x < -1.0) return __builtin_nanf("");
    if (x == 1.0) return (float)PI_2_D;
    if (x == -1.0) return (float)(-PI_2_D);
    return (float)atan(x / __builtin_sqrt((1.0 - x) * (1.0 + x)));
}

// (double)a / REF_PI, correctly rounded, for a float a, without the divide sequence:
// q = RN(a y) with y = RN(1/pi) is within 1 ulp of the quotient, r = a - q pi is exact in one
// fma, and RN(q + r y) is the correctly rounded quotient (Markstein's theorem; pi's
// significand is not all ones).  a = +-0 returns q itself (keeps the zero's sign).
// tests/test_exact_identities.py checks it against the IEEE divide for every float in
// [-2, 2] (asinf_ returns |a| <= pi/2; atanf_ / 2 returns |a| <= pi/4).
__device__ __forceinline__ double div_pi(float a) {
    constexpr double INV_PI = 1.0 / REF_PI;
    const double q = (double)a * INV_PI;
    if (q == 0.0) return q;
    const double r = __builtin_fma(-q, REF_PI, (double)a);
    return __builtin_fma(r, INV_PI, q);
}

// (float)k / 255.0f for an integer 0 <= k <= 255: the exact-quotient rule of qdiv
// (cpt_device.hpp) with the double reciprocal of 255 (every k/255 > 0 is a normal float, and
// 0 gives +0), checked for all 256 k in tests/test_exact_identities.py.
__device__ __forceinline__ float div255(uint32_t k) {
    return (float)((double)k * (1.0 / 255.0));
}

}  // namespace dm

// ------------------------------------------------------------------------------------
// Short forms of the BSDF lobe's transcendentals (round 6).  Each returns a double within
// ~2^-49 (relative) of the exact function, and `ok`: whether that double rounds to the same
// float as every double within 2^-43 of it -- then it rounds like the full dm:: sequence
// (itself within ~2^-51 of the exact value), and the caller uses it; otherwise (about 1 in
// 2^18 inputs, and every input outside the form's domain) the caller runs the dm:: sequence.
// Tables and constants: cpt_fm_tables.hpp (tools/make_fastmath_tables.py).  Checked on the
// device against the dm:: sequence for every float of the lobe's domain
// (test_gpu_parity.py::test_lobe_*_exhaustive) and restated on the host against the oracle
// (tests/test_fastmath.py).
// ------------------------------------------------------------------------------------
namespace fm {

__device__ const double g_log_tab[2 * FM_LOG_N] = CPT_FM_LOG_TABLE_INIT;        // {c_i, -ln c_i}
__device__ const double g_exp_tab[FM_EXP_N] = CPT_FM_EXP_TABLE_INIT;             // 2^(j/N)
__device__ const double g_sc_tab[2 * (2 * FM_SC_N + 1)] = CPT_FM_SC_TABLE_INIT;  // {sin, cos}(k pi/32)

// d rounds to float like every double within 2^-43 |d| of it, and 2^-126 <= |d| < 2: d's 29
// bits below float precision (all in its low word) are not within 2^10 double ulps of the
// half-way pattern 2^28 (2^10 ulps >= 2^-43 |d|).  NaN, inf, 0 and subnormal floats fail.
__device__ __forceinline__ bool sure_f32(double d) {
    const uint32_t lo = (uint32_t)__double2loint(d), hi = (uint32_t)__double2hiint(d) & 0x7fffffffu;
    const int dm_ = (int)(lo & 0x1fffffffu) - (1 << 28);
    return hi - 0x38100000u < 0x07f00000u && (dm_ >= 1024 || dm_ <= -1024);
}

// pow(x, y) for a float x in [2^-126, 1] and 0 < y <= 1 with |y ln x| <= 2 (else ok = false):
// x = 2^e m, ln x = e ln2 - ln c_i + log1p(m c_i - 1) (i: m's top 7 fraction bits; the fma is
// exact), then exp(t) = 2^(n/128) P(s) with n = round(t 128/ln2) (the 1.5 2^52 shifter: n is
// the low word), s the remainder in units of ln2/128, 2^(n>>7) applied to T_j's exponent field.
__device__ __forceinline__ double pow_unit(float x, double y, bool& ok) {
    const uint32_t ux = __float_as_uint(x);
    const int e = (int)(ux >> 23) - 127;
    const uint32_t i = (ux >> 16) & (uint32_t)(FM_LOG_N - 1);
    const double m = (double)__uint_as_float((ux & 0x007fffffu) | 0x3f800000u);
    const double c = g_log_tab[2 * i], lnc = g_log_tab[2 * i + 1];
    const double r = __builtin_fma(m, c, -1.0);
    double q = __builtin_fma(r, dm::kc(FM_L6), dm::kc(FM_L5));
    q = __builtin_fma(r, q, dm::kc(FM_L4));
    q = __builtin_fma(r, q, dm::kc(FM_L3));
    q = __builtin_fma(r, q, dm::kc(FM_L2));
    const double lp = __builtin_fma(r * r, q, r);
    const double t = y * __builtin_fma((double)e, dm::kc(FM_LN2), lnc + lp);
    constexpr double SHIFT = 0x1.8p52;
    const double tt = __builtin_fma(t, dm::kc(FM_KN_HI), SHIFT);
    const double nd = tt - SHIFT;
    const int n = __double2loint(tt);
    double s = __builtin_fma(t, dm::kc(FM_KN_HI), -nd);
    s = __builtin_fma(t, dm::kc(FM_KN_LO), s);
    double p = __builtin_fma(s, dm::kc(FM_E4), dm::kc(FM_E3));
    p = __builtin_fma(s, p, dm::kc(FM_E2));
    p = __builtin_fma(s, p, dm::kc(FM_E1));
    p = __builtin_fma(s, p, 1.0);
    const double T = g_exp_tab[n & (FM_EXP_N - 1)];
    const double Ts = __hiloint2double(__double2hiint(T) + (int)((uint32_t)(n >> 7) << 20), __double2loint(T));
    const double d = Ts * p;
    ok = ux - 0x00800000u <= 0x3f000000u && y > 0.0 && y <= 1.0 && t >= -2.0 && sure_f32(d);
    return d;
}

// sin and cos of a float phi in [0, 2 pi] (else ok = false): k = round(phi 32/pi), r = phi -
// k pi/32 (two-part constant: exact to ~2^-53 |r|), sin phi = S_k cos r + C_k sin r, cos phi =
// C_k cos r - S_k sin r; the table's zeros and ones are exact, so each result near a zero of sin
// or cos is the short series of r alone.
__device__ __forceinline__ void sincos_2pi(float phi, double& s, double& c, bool& ok) {
    const double x = (double)phi;
    constexpr double SHIFT = 0x1.8p52;
    const double tt = __builtin_fma(x, dm::kc(FM_SC_K), SHIFT);
    const double kd = tt - SHIFT;
    const uint32_t k = (uint32_t)__double2loint(tt);
    double r = __builtin_fma(-kd, dm::kc(FM_SC_P1), x);
    r = __builtin_fma(-kd, dm::kc(FM_SC_P2), r);
    const double r2 = r * r;
    double ps = __builtin_fma(r2, dm::kc(FM_S7), dm::kc(FM_S5));
    ps = __builtin_fma(r2, ps, dm::kc(FM_S3));
    const double sr = __builtin_fma(r * r2, ps, r);
    double pc = __builtin_fma(r2, dm::kc(FM_C6), dm::kc(FM_C4));
    pc = __builtin_fma(r2, pc, dm::kc(FM_C2));
    const double cr = __builtin_fma(r2, pc, 1.0);
    const uint32_t kk = k <= (uint32_t)(2 * FM_SC_N) ? k : 0u;
    const double S = g_sc_tab[2 * kk], C = g_sc_tab[2 * kk + 1];
    s = __builtin_fma(S, cr, C * sr);
    c = __builtin_fma(C, cr, -(S * sr));
    ok = phi >= 0.0f && phi <= 6.28318548f && sure_f32(s) && sure_f32(c);
}

__device__ const double g_at_tab[2 * (FM_AT_N + 1)] = CPT_FM_AT_TABLE_INIT;   // {atan(k/32), pi/2 - atan(k/32)}

// atan(n / m) for n >= 0, m > 0 (else ok = false): with k = round(32 min(n/m, m/n)) from a float
// estimate and c = k/32, atan(n/m) = A_k + atan((n - c m) / (m + c n)) when n <= m, and
// B_k - atan((m - c n) / (n + c m)) when n > m (A_k = atan c, B_k = pi/2 - atan c); each
// numerator and denominator is one fma (the numerator's cancellation is exact inside it), the
// quotient a reciprocal (v_rcp_f64 + two Newton steps) times the numerator, |d| <= 2^-6, and
// atan d to d^7.  No IEEE divide: the quotient n/m itself is never formed.
__device__ __forceinline__ double atan_ratio(double n, double m, bool& ok) {
    const bool big = n > m;
    const float rf = (float)(big ? m : n) * __builtin_amdgcn_rcpf((float)(big ? n : m));
    const float kf = __builtin_fminf(__builtin_rintf(32.0f * rf), 32.0f);
    const double c = (double)kf * 0.03125;
    const double num = big ? __builtin_fma(-c, n, m) : __builtin_fma(-c, m, n);
    const double den = big ? __builtin_fma(c, m, n) : __builtin_fma(c, n, m);
    double r = __builtin_amdgcn_rcp(den);
    double e = __builtin_fma(-den, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-den, r, 1.0);
    r = __builtin_fma(r, e, r);
    const double d = num * r;
    const double d2 = d * d;
    double p = __builtin_fma(d2, dm::kc(FM_A7), dm::kc(FM_A5));
    p = __builtin_fma(d2, p, dm::kc(FM_A3));
    const double at = __builtin_fma(d * d2, p, d);
    const int k = (int)kf;   // 0..32 (a NaN estimate: the guard below fails)
    const double T = g_at_tab[2 * (k >= 0 && k <= FM_AT_N ? k : 0) + (big ? 1 : 0)];
    const double res = big ? T - at : T + at;
    ok = n >= 0.0 && m > 0.0 && sure_f32(res);
    return res;
}

}  // namespace fm

// Miss's atanf(d.y / d.x) (path_tracer.cu:120): (float)dm::atan((double)x) through fm::atan_ratio
// (|x| over 1), the full sequence where its guard fails (test_miss_atan_asin_exhaustive).
__device__ __forceinline__ float miss_atanf(float x) {
    bool ok;
    const double a = fm::atan_ratio(__builtin_fabs((double)x), 1.0, ok);
    float f = (float)(x < 0.0f ? -a : a);
    if (__builtin_expect(!ok, 0)) f = dm::atanf_(x);
    return f;
}

// Miss's asinf(d.z) (path_tracer.cu:119): dm::asinf_ is (float)atan(z / sqrt((1 - z)(1 + z)));
// fm::atan_ratio takes |z| over the same square root directly, so neither the quotient's divide
// nor a second atan reduction runs; the full sequence where the guard fails (z = +-1, 0, NaN).
__device__ __forceinline__ float miss_asinf(float z) {
    const double x = (double)z;
    bool ok;
    const double a = fm::atan_ratio(__builtin_fabs(x), __builtin_sqrt((1.0 - x) * (1.0 + x)), ok);
    float f = (float)(z < 0.0f ? -a : a);
    if (__builtin_expect(!ok, 0)) f = dm::asinf_(z);
    return f;
}

// The lobe's z = (float)pow(x_1, inv_alpha) (material.cu:24,45,78,85,104): Diffuse's exponent 1/2
// as sqrtf -- (float)dm::pow(x, 0.5) == sqrtf(x) for every float x in [2^-42, 1] (x_1 >= 2^-33),
// checked on the host against the oracle and on the device (test_lobe_pow_exhaustive); the
// other exponents through fm::pow_unit, the dm:: sequence where its guard fails.
__device__ __forceinline__ float lobe_pow(float x, double y) {
    if (y == 0.5 && x >= 0x1p-42f) return sqrt_nn(x);
    bool ok;
    const double d = fm::pow_unit(x, y, ok);
    float z = (float)d;
    if (__builtin_expect(!ok, 0)) z = (float)dm::pow((double)x, y);
    return z;
}

// sinf / cosf of the lobe's phi = (float)(2 pi x_2) in [0, 2 pi] (material.cu:26-27,47-48):
// fm::sincos_2pi, dm::sincosf_ where its guard fails (test_lobe_sincos_exhaustive).
__device__ __forceinline__ void lobe_sincos(float phi, float* s_out, float* c_out) {
    double s, c;
    bool ok;
    fm::sincos_2pi(phi, s, c, ok);
    *s_out = (float)s;
    *c_out = (float)c;
    if (__builtin_expect(!ok, 0)) dm::sincosf_(phi, s_out, c_out);
}

// ------------------------------------------------------------------------------------
// cuRAND XORWOW (curand_kernel.h restated).  State lives in registers
// for a whole render; HBM holds it planar [6][npix] between renders.
// ------------------------------------------------------------------------------------
struct Xorwow { uint32_t v0, v1, v2, v3, v4, d; };

__device__ __forceinline__ uint32_t xorwow_next(Xorwow& s) {
    uint32_t t = s.v0 ^ (s.v0 >> 2);
    s.v0 = s.v1; s.v1 = s.v2; s.v2 = s.v3; s.v3 = s.v4;
    s.v4 = (s.v4 ^ (s.v4 << 4)) ^ (t ^ (t << 1));
    s.d += 362437u;
    return s.v4 + s.d;
}

// curand_uniform: x * 2^-32 + 2^-33 (the product is exact; result in (0, 1]).
__device__ __forceinline__ float uniform(Xorwow& s) {
    uint32_t x = xorwow_next(s);
    return (float)x * 2.3283064e-10f + (2.3283064e-10f / 2.0f);
}

// ------------------------------------------------------------------------------------
// Scene data in HBM (DESIGN.md §The path and its boundary)
// ------------------------------------------------------------------------------------
// BVH node, 32 B, right-first preorder ("skip-link" order): the node after n in memory is
// its right child (the child the reference's DFS pops first, bvh.cu:201-202).  The eight
// octant orders (CPT_TRAVERSAL_ORDERED) put the near child of each split first instead.
//   internal (code < 0): a = AABB min, b = AABB max, miss = next node once n's subtree is
//            skipped or finished
//   leaf     (code >= 0): the primitive inline (a leaf's own box is never tested: in the
//            reference its slab test only decides whether to push two -1 sentinels):
//            a = center, b = {radius, y_pos, height}, code = material << 2 | type
//            (type 3 = unknown PrimitiveType: IntersectionTest returns false, object.cu:126);
//            the walk continues at n + 1, and miss = the leaf's position in the reference
//            order (its rank for equal hit distances)
struct __attribute__((aligned(16))) Node {
    float a0, a1, a2;
    int32_t miss;
    float b0, b1, b2;
    int32_t code;
};
static_assert(sizeof(Node) == 32, "Node is 32 B");

// Material, 48 B: Material (material.h:17-35) reduced to what the shaders read, prepared once
// per material on the device (k_prepare_materials):
//   att   = GetKd(0, 0) (material.cu:11-18): kd_, or a textured material's (0, 0) sample
//   rad   = emit_intensity_ * kd_ (material.cu:36,62,97,141); in a textured material kd_
//           aliases tex_, so these are the handle's bits, as in the reference's union
//   inv_alpha = 1.0 / (double)powf(1000, smoothness_) (material.cu:43,69,103)
//   inv_ior = 1.f / ior_, and for Glass schlick_r0 = ((1 - ior_) / (1 + ior_))^2 in the
//   reflectivity slot (ray_tracing_math.hpp:65-67, material.cu:114-133): the shader's own
//   quotients, computed once per material instead of once per hit
// The host stages {att = kd_ bits, rad.x = emit_intensity_, smoothness} and the kernel
// completes it.
struct __attribute__((aligned(16))) Mat {
    float att_x, att_y, att_z;
    int32_t type;
    float rad_x, rad_y, rad_z;
    float ior;
    union { float reflectivity; float schlick_r0; };   // Mirror: reflectivity_; Glass: r0
    union { float smoothness; float inv_ior; };        // staged: smoothness_; prepared: 1 / ior
    double inv_alpha;
};
static_assert(sizeof(Mat) == 48, "Mat is 48 B");

// A material texture bound with cpt_bind_texture: packed RGBA8 words, `cols` valid columns.
struct TexDesc {
    const uint32_t* texels;
    int32_t w, h, cols, addr, filter, pad_;
};
static_assert(sizeof(TexDesc) == 32, "TexDesc is 32 B");

struct Ray { v3 o, d; float tmin, tmax; };

// ------------------------------------------------------------------------------------
// Exact f32 quotients through a per-ray double reciprocal.
//
// qdiv_raw(a, y) with y = RN_f64(1 / (double)d) equals RN_f32(a / d), the IEEE f32 quotient,
// whenever that quotient is a normal number, infinite, NaN, or a is +-0:
//   * (double)a and y are exact / correctly rounded, so the product has relative error
//     < 2^-52 before the final rounding to f32;
//   * a quotient of two 24-bit significands in the normal range is never a f32 rounding
//     midpoint (the product of an odd 25-bit and a 24-bit integer has >= 25 significant
//     bits) and is >= 2^-50 (relative) away from every midpoint, so the double result rounds
//     to the same f32 (the innocuous double-rounding bound p' >= 2p + 2 for division);
//   * d = +-0 gives y = +-inf and a*y = +-inf / NaN exactly as a/d.
// Subnormal (and underflowed-to-zero) quotients CAN sit exactly on a midpoint (d with few
// significant bits), where the rounded reciprocal breaks the tie the wrong way; qdiv() and
// the slab test fall back to the IEEE divide whenever |q| < 2^-126.  k_selftest_qdiv checks
// qdiv against v_div_* on 4.3e9 hashed pairs per operand family.
// One reciprocal per ray and axis replaces the 11-instruction IEEE divide sequence per slab
// plane and per intersector root.
// ------------------------------------------------------------------------------------
constexpr float FLT_MIN_NORMAL = 1.17549435e-38f;   // 2^-126

// 1.0 / (double)d, correctly rounded, in 5 f64 ops instead of the 11-op IEEE divide: v_rcp_f64
// and two Newton steps give the correctly rounded reciprocal of every finite nonzero float
// (checked for all 2^32 patterns by tools/exact_rcp_check.hip and test_rcp_d_exhaustive);
// for +-0 and +-inf the steps make a NaN and v_rcp_f64's own +-inf / +-0 is the IEEE result.
__device__ __forceinline__ double rcp_d(float d) {
    const double x = (double)d;
    const double r0 = __builtin_amdgcn_rcp(x);
    double e = __builtin_fma(-x, r0, 1.0);
    double r = __builtin_fma(r0, e, r0);
    e = __builtin_fma(-x, r, 1.0);
    r = __builtin_fma(r, e, r);
    return r == r ? r : r0;
}
__device__ __forceinline__ float qdiv_raw(float a, double y) { return (float)((double)a * y); }

__device__ __forceinline__ float qdiv(float a, float d, double y) {
    float q = qdiv_raw(a, y);
    if (__builtin_expect(__builtin_fabsf(q) < FLT_MIN_NORMAL, 0)) q = a / d;
    return q;
}

}  // namespace cpt
