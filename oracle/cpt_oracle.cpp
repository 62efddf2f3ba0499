// cpt_oracle.cpp — TEST INFRASTRUCTURE ONLY (the parity checker / CPU baseline).
//
// Scalar C++ restatement of DearPoca/CppPathTracer's per-pixel Monte-Carlo integrator
// (reference @ /root/reference).  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load this library.  The product (cpppathtracer_amd/, libcpt.so)
// never includes, links or calls anything under oracle/.
//
// Parity status:
//   * The reference ships no tests, fixtures or golden vectors and
//     cannot be compiled here (CUDA 11.7 + cuRAND + OpenCV + Win32).  Pinned in-container:
//       - XORWOW transition and the 2^67 subsequence jump: checked against rocRAND's
//         precomputed tables (tests/test_oracle_rng.py);
//       - the sky texture bytes (PIL decode == lossless PNG decode, tools/make_sky_fixture.py).
//     UNPINNED (no reference artefact exists): cuRAND's curand_init salts/multipliers and
//     uniform mapping (recalled from the public curand_kernel.h), CUDA libdevice
//     transcendental rounding, NVIDIA TMU bilinear weight quantisation.  These are defined
//     here as documented deterministic choices and the HIP path must match them bit-exactly.
//
// Build: see oracle/Makefile (g++ -O2 -ffp-contract=off; no fast-math, no FMA contraction).

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

namespace {

// ---------------------------------------------------------------------------------------
// Reference POD layouts (restated; byte offsets checked by static_asserts and by tests).
// ---------------------------------------------------------------------------------------
struct f3 { float x, y, z; };                                   // CUDA float3, 12 B

struct Material {                                               // material.h:17-35 (40 B)
    int32_t type;            // MaterialType::Enum  @0
    uint8_t have_tex;        // bool                @4
    uint8_t pad_[3];
    union { f3 kd; uint64_t tex; } u;  //           @8 (16 B, align 8)
    float refractive_index;  //                     @24
    float emit_intensity;    //                     @28
    float smoothness;        //                     @32
    float reflectivity;      //                     @36
};
static_assert(sizeof(Material) == 40, "Material layout");

struct Object {                                                 // object.h:17-32 (72 B)
    int32_t type;            // PrimitiveType::Enum @0
    int32_t pad_;
    Material material;       //                     @8
    f3 center;               //                     @48
    float radius;            //                     @60
    float y_pos;             //                     @64
    float height;            //                     @68
};
static_assert(sizeof(Object) == 72, "Object layout");

struct Camera {                                                 // motional_camera.h:8-24 (136 B)
    f3 vup;                  // @0
    int32_t width, height;   // @12, @16
    uint32_t cur_sample_idx; // @20
    f3 origin, look_at;      // @24, @36
    float view_fov, dist_to_focus, lens_radius, move_speed;  // @48..@60
    f3 u, v, w;              // @64, @76, @88
    f3 top_left, horizontal, vertical;                       // @100, @112, @124
};
static_assert(sizeof(Camera) == 136, "MotionalCamera layout");

enum { PRIM_SPHERE = 0, PRIM_PLATFORM = 1, PRIM_CYLINDER = 2 };          // object.h:7-15
enum { MAT_DIFFUSE = 0, MAT_METAL = 1, MAT_MIRROR = 2, MAT_GLASS = 3 };  // material.h:5-15

const float DEFAULT_RAY_TMAX = 1e30f;   // ray_tracing_common.h:11
const float BOUNCE_RAY_TMIN = 2e-5f;    // ray_tracing_common.h:12
const uint32_t MAX_RECURSION_DEPTH_SET = 32;  // path_tracer.h:13
const double REF_PI = 3.14159265358979323846;  // ray_tracing_math.hpp:11-13 (M_PI, double)

// MIN/MAX/ABS are ternary macros in the reference (ray_tracing_math.hpp:15-26): NaN-sensitive.
inline float MIN_(float a, float b) { return a < b ? a : b; }
inline float MAX_(float a, float b) { return a > b ? a : b; }
inline float ABS_(float a) { return a >= 0 ? a : -a; }

// ---------------------------------------------------------------------------------------
// helper_math.h host-path semantics (Common/helper_math.h, lines cited per op).
// ---------------------------------------------------------------------------------------
inline f3 mk(float x, float y, float z) { return f3{x, y, z}; }
inline f3 mk1(float s) { return f3{s, s, s}; }                                  // :135-138
inline f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
inline f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
inline f3 mul(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
inline f3 mul(float s, f3 a) { return mk(s * a.x, s * a.y, s * a.z); }          // :834-837
inline f3 mul(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
inline f3 divs(f3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }         // :1013-1016
inline f3 neg(f3 a) { return mk(-a.x, -a.y, -a.z); }
inline float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }      // :1264-1267
inline float length(f3 v) { return sqrtf(dot(v, v)); }                          // :1307-1310
inline f3 normalize(f3 v) { float inv = 1.0f / sqrtf(dot(v, v)); return mul(v, inv); }  // :1325-1329, host rsqrtf :78-81
inline f3 cross(f3 a, f3 b) {                                                   // :1436-1439
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
inline f3 reflect(f3 i, f3 n) { return sub(i, mul(mul(2.0f, n), dot(n, i))); }   // :1427-1430

// ---------------------------------------------------------------------------------------
// Deterministic transcendentals ("detmath").  The reference calls CUDA libdevice pow / sinf /
// cosf / asinf / atanf (material.cu:24-25,44-46,70,78,86,105; path_tracer.cu:119;
// ray_tracing_math.hpp:68).  libdevice is not available, so the reference semantics are
// defined here as: evaluate in double with these exact operation sequences (error well
// under 1e-15 relative), then round as the C++ expression does.  The HIP kernels implement
// the identical sequences: the polynomial steps are explicit fused multiply-adds (std::fma
// here, v_fma_f64 there) and FMA contraction is off everywhere else, so the results are equal
// bit for bit.  Accuracy vs glibc is checked by tests/test_oracle_math.py.
// ---------------------------------------------------------------------------------------
inline uint64_t dbits(double x) { uint64_t u; std::memcpy(&u, &x, 8); return u; }
inline double bitsd(uint64_t u) { double x; std::memcpy(&x, &u, 8); return x; }

const double LN2_HI = 6.93147180369123816490e-01;   // 0x3fe62e42fee00000 (trailing zeros)
const double LN2_LO = 1.90821492927058770002e-10;   // 0x3dea39ef35793c76
const double INV_LN2 = 1.44269504088896338700e+00;
const double SQRT2 = 1.41421356237309514547e+00;

double dm_log(double x) {
    if (!(x > 0.0)) {                       // x <= 0 or NaN
        if (x == 0.0) return -INFINITY;
        return NAN;
    }
    if (x == INFINITY) return INFINITY;
    uint64_t u = dbits(x);
    int e = (int)((u >> 52) & 0x7ff);
    if (e == 0) {                           // subnormal: scale by 2^54
        x = x * 18014398509481984.0;
        u = dbits(x);
        e = (int)((u >> 52) & 0x7ff) - 54;
    }
    e -= 1023;
    double m = bitsd((u & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL);  // [1,2)
    if (m > SQRT2) { m = m * 0.5; e += 1; }
    double f = m - 1.0;
    double s = f / (2.0 + f);
    double s2 = s * s;
    // 2*atanh(s) = 2s(1 + s2/3 + s2^2/5 + ...), |s| <= 0.1716, 12 terms
    double p = 1.0 / 25.0;
    p = std::fma(s2, p, 1.0 / 23.0);
    p = std::fma(s2, p, 1.0 / 21.0);
    p = std::fma(s2, p, 1.0 / 19.0);
    p = std::fma(s2, p, 1.0 / 17.0);
    p = std::fma(s2, p, 1.0 / 15.0);
    p = std::fma(s2, p, 1.0 / 13.0);
    p = std::fma(s2, p, 1.0 / 11.0);
    p = std::fma(s2, p, 1.0 / 9.0);
    p = std::fma(s2, p, 1.0 / 7.0);
    p = std::fma(s2, p, 1.0 / 5.0);
    p = std::fma(s2, p, 1.0 / 3.0);
    double r = std::fma(2.0 * s, s2 * p, 2.0 * s);
    double de = (double)e;
    return std::fma(de, LN2_HI, std::fma(de, LN2_LO, r));
}

double dm_ldexp(double x, int k) {
    // x in [0.5, 2], k in [-1100, 1100]; two-step scaling keeps every step exact until the
    // final (possibly subnormal) multiply.
    if (k > 1023) { x = x * bitsd(0x7fe0000000000000ULL); k -= 1023; if (k > 1023) k = 1023; }
    if (k < -1022) { x = x * bitsd(0x0010000000000000ULL); k += 1022; if (k < -1022) k = -1022; }
    return x * bitsd((uint64_t)(k + 1023) << 52);
}

double dm_exp(double x) {
    if (x != x) return x;
    if (x > 709.782712893384) return INFINITY;
    if (x < -745.1332191019412) return 0.0;
    double k = floor(std::fma(x, INV_LN2, 0.5));
    double r = std::fma(-k, LN2_LO, std::fma(-k, LN2_HI, x));   // |r| <= 0.3466
    // Taylor to r^13
    double p = 1.0 / 6227020800.0;              // 1/13!
    p = std::fma(r, p, 1.0 / 479001600.0);              // 1/12!
    p = std::fma(r, p, 1.0 / 39916800.0);
    p = std::fma(r, p, 1.0 / 3628800.0);
    p = std::fma(r, p, 1.0 / 362880.0);
    p = std::fma(r, p, 1.0 / 40320.0);
    p = std::fma(r, p, 1.0 / 5040.0);
    p = std::fma(r, p, 1.0 / 720.0);
    p = std::fma(r, p, 1.0 / 120.0);
    p = std::fma(r, p, 1.0 / 24.0);
    p = std::fma(r, p, 1.0 / 6.0);
    p = std::fma(r, p, 0.5);
    p = std::fma(r, p, 1.0);
    p = std::fma(r, p, 1.0);
    return dm_ldexp(p, (int)k);
}

// pow(double, double) with the C99 special cases the integrator can reach.
double dm_pow(double x, double y) {
    if (y == 0.0) return 1.0;
    if (x == 1.0) return 1.0;
    if (x != x || y != y) return NAN;
    if (x == 0.0) return y > 0.0 ? 0.0 : INFINITY;
    if (x < 0.0) {
        double yi = floor(y);
        if (yi != y) return NAN;
        double m = dm_exp(y * dm_log(-x));
        double half = y * 0.5;
        return (floor(half) != half) ? -m : m;   // odd integer exponent keeps the sign
    }
    if (x == INFINITY) return y > 0.0 ? INFINITY : 0.0;
    return dm_exp(y * dm_log(x));
}

float dm_powf(float x, float y) { return (float)dm_pow((double)x, (double)y); }

// pow(x, 5) of schlick (ray_tracing_math.hpp:68, an integer exponent): x^2 exact in double, then
// two rounded products; the device's dm::pow5f is the same sequence.
float dm_pow5f(float xf) {
    const double x = (double)xf;
    const double x2 = x * x;
    return (float)(x2 * x2 * x);
}

// pi/2 split (fdlibm constants): PIO2_1 has 33 significant bits.
const double PIO2_1 = 1.57079632673412561417e+00;
const double PIO2_2 = 6.07710050650619224932e-11;
const double PIO2_3 = 2.02226624879595063154e-21;
const double TWO_OVER_PI = 6.36619772367581382433e-01;

double dm_sin_poly(double r) {   // |r| <= pi/4, Taylor to r^19
    double r2 = r * r;
    double p = -1.0 / 121645100408832000.0;     // -1/19!
    p = std::fma(r2, p, 1.0 / 355687428096000.0);       // 1/17!
    p = std::fma(r2, p, -1.0 / 1307674368000.0);        // -1/15!
    p = std::fma(r2, p, 1.0 / 6227020800.0);            // 1/13!
    p = std::fma(r2, p, -1.0 / 39916800.0);             // -1/11!
    p = std::fma(r2, p, 1.0 / 362880.0);
    p = std::fma(r2, p, -1.0 / 5040.0);
    p = std::fma(r2, p, 1.0 / 120.0);
    p = std::fma(r2, p, -1.0 / 6.0);
    return std::fma(r, r2 * p, r);
}

double dm_cos_poly(double r) {   // |r| <= pi/4, Taylor to r^20
    double r2 = r * r;
    double p = 1.0 / 2432902008176640000.0;     // 1/20!
    p = std::fma(r2, p, -1.0 / 6402373705728000.0);     // -1/18!
    p = std::fma(r2, p, 1.0 / 20922789888000.0);        // 1/16!
    p = std::fma(r2, p, -1.0 / 87178291200.0);          // -1/14!
    p = std::fma(r2, p, 1.0 / 479001600.0);             // 1/12!
    p = std::fma(r2, p, -1.0 / 3628800.0);
    p = std::fma(r2, p, 1.0 / 40320.0);
    p = std::fma(r2, p, -1.0 / 720.0);
    p = std::fma(r2, p, 1.0 / 24.0);
    p = std::fma(r2, p, -0.5);
    return std::fma(r2, p, 1.0);
}

// Shared range reduction; returns quadrant in *q.
double dm_reduce(double x, int* q) {
    double k = floor(std::fma(x, TWO_OVER_PI, 0.5));
    double r = std::fma(-k, PIO2_3, std::fma(-k, PIO2_2, std::fma(-k, PIO2_1, x)));
    double km = k - 4.0 * floor(k * 0.25);     // k mod 4 in [0,4)
    *q = (int)km;
    return r;
}

float dm_sinf(float xf) {
    double x = (double)xf;
    if (x != x || x == INFINITY || x == -INFINITY) return NAN;
    int q;
    double r = dm_reduce(x, &q);
    double s;
    switch (q) {
        case 0: s = dm_sin_poly(r); break;
        case 1: s = dm_cos_poly(r); break;
        case 2: s = -dm_sin_poly(r); break;
        default: s = -dm_cos_poly(r); break;
    }
    return (float)s;
}

float dm_cosf(float xf) {
    double x = (double)xf;
    if (x != x || x == INFINITY || x == -INFINITY) return NAN;
    int q;
    double r = dm_reduce(x, &q);
    double c;
    switch (q) {
        case 0: c = dm_cos_poly(r); break;
        case 1: c = -dm_sin_poly(r); break;
        case 2: c = -dm_cos_poly(r); break;
        default: c = dm_sin_poly(r); break;
    }
    return (float)c;
}

const double PI_2_D = 1.57079632679489655800e+00;  // pi/2 rounded to double

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

double dm_atan(double t) {
    // fdlibm's reduction to |x| < 7/16 around atan(0.5), atan(1), atan(1.5), atan(inf), with
    // one division chosen by selects, and its odd/even split of an 11-term minimax polynomial
    // (DESIGN.md §Numerics).  Identical operation sequence on the device (cpt_device.hpp dm::atan).
    if (t != t || t == 0.0) return t;
    const double sgn = t < 0.0 ? -1.0 : 1.0;
    const double a = t < 0.0 ? -t : t;
    if (a == INFINITY) return sgn * PI_2_D;
    const bool r0 = a < 0.4375, r1 = a < 0.6875, r2 = a < 1.1875, r3 = a < 2.4375;
    const double num = r0 ? a : r1 ? 2.0 * a - 1.0 : r2 ? a - 1.0 : r3 ? a - 1.5 : -1.0;
    const double den = r0 ? 1.0 : r1 ? 2.0 + a : r2 ? a + 1.0 : r3 ? 1.0 + 1.5 * a : a;
    const double hi = r1 ? ATAN_HI0 : r2 ? ATAN_HI1 : r3 ? ATAN_HI2 : ATAN_HI3;
    const double lo = r1 ? ATAN_LO0 : r2 ? ATAN_LO1 : r3 ? ATAN_LO2 : ATAN_LO3;
    const double x = num / den;
    const double z = x * x, w = z * z;
    const double s1 = z * std::fma(w, std::fma(w, std::fma(w, std::fma(w, std::fma(w, AT10, AT8), AT6), AT4), AT2), AT0);
    const double s2 = w * std::fma(w, std::fma(w, std::fma(w, std::fma(w, AT9, AT7), AT5), AT3), AT1);
    const double r = r0 ? std::fma(-x, s1 + s2, x) : hi - (std::fma(x, s1 + s2, -lo) - x);
    return sgn * r;
}

float dm_atanf(float x) { return (float)dm_atan((double)x); }

float dm_asinf(float xf) {
    double x = (double)xf;
    if (x != x) return NAN;
    if (x > 1.0 || x < -1.0) return NAN;
    if (x == 1.0) return (float)PI_2_D;
    if (x == -1.0) return (float)(-PI_2_D);
    return (float)dm_atan(x / sqrt((1.0 - x) * (1.0 + x)));
}

// ---------------------------------------------------------------------------------------
// cuRAND XORWOW restatement (ray_tracing_math.hpp:82-104 call sites; the algorithm lives in
// CUDA 11.7 curand_kernel.h, not present here).  State: v[5], d.  Layout in this library's
// buffers is planar [6][npix]: v0..v4, d.
// ---------------------------------------------------------------------------------------
struct Xorwow { uint32_t v[5]; uint32_t d; };

inline uint32_t xorwow_next(Xorwow& s) {                       // curand(): xorshift + Weyl
    uint32_t t = s.v[0] ^ (s.v[0] >> 2);
    s.v[0] = s.v[1]; s.v[1] = s.v[2]; s.v[2] = s.v[3]; s.v[3] = s.v[4];
    s.v[4] = (s.v[4] ^ (s.v[4] << 4)) ^ (t ^ (t << 1));
    s.d += 362437u;
    return s.v[4] + s.d;
}

// curand_uniform: x * CURAND_2POW32_INV + CURAND_2POW32_INV/2, in (0, 1].
// 2.3283064e-10f rounds to exactly 2^-32, so the product is exact and FMA contraction
// (nvcc default) cannot change the result.
inline float uniform(Xorwow& s) {
    uint32_t x = xorwow_next(s);
    return (float)x * 2.3283064e-10f + (2.3283064e-10f / 2.0f);
}

// Linear part of one XORWOW step as a 160x160 GF(2) matrix stored column-wise in rocRAND's
// layout m[(word*32 + bit)*5 + k] (rocrand_xorwow.h:51-65): column (word,bit) = A * e(word,bit).
struct BitMat { uint32_t m[800]; };

void matvec(const BitMat& M, const uint32_t in[5], uint32_t out[5]) {
    uint32_t r[5] = {0, 0, 0, 0, 0};
    for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 32; ++j)
            if (in[i] & (1u << j))
                for (int k = 0; k < 5; ++k) r[k] ^= M.m[(i * 32 + j) * 5 + k];
    std::memcpy(out, r, sizeof(r));
}

BitMat matmul(const BitMat& A, const BitMat& B) {   // A*B
    BitMat C;
    for (int c = 0; c < 160; ++c) matvec(A, &B.m[c * 5], &C.m[c * 5]);
    return C;
}

struct JumpTables {
    BitMat seq[64];     // seq[t] = A^(2^67 * 2^t)
};

const JumpTables& jump_tables() {
    static JumpTables* tbl = nullptr;
    static std::once_flag once;
    std::call_once(once, [] {
        tbl = new JumpTables;
        BitMat A;
        for (int c = 0; c < 160; ++c) {
            Xorwow s{};
            s.v[c / 32] = 1u << (c % 32);
            xorwow_next(s);
            std::memcpy(&A.m[c * 5], s.v, 20);
        }
        BitMat P = A;
        for (int i = 0; i < 67; ++i) P = matmul(P, P);      // A^(2^67)
        tbl->seq[0] = P;
        for (int t = 1; t < 64; ++t) tbl->seq[t] = matmul(tbl->seq[t - 1], tbl->seq[t - 1]);
    });
    return *tbl;
}

// curand_init(seed, subsequence, offset=0, &state) — curand_kernel.h (CUDA 11.7)
// _curand_init_scratch.  Salts / multipliers recalled from the public header (UNPINNED).
Xorwow curand_init(uint64_t seed, uint64_t subsequence) {
    uint32_t s0 = (uint32_t)seed ^ 0xaad26b49u;
    uint32_t s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
    uint32_t t0 = 1099087573u * s0;
    uint32_t t1 = 2591861531u * s1;
    Xorwow st;
    st.d = 6615241u + t1 + t0;
    st.v[0] = 123456789u + t0;
    st.v[1] = 362436069u ^ t0;
    st.v[2] = 521288629u + t1;
    st.v[3] = 88675123u ^ t1;
    st.v[4] = 5783321u + t0;
    const JumpTables& J = jump_tables();
    for (int t = 0; t < 64; ++t)
        if ((subsequence >> t) & 1ull) matvec(J.seq[t], st.v, st.v);
    // d unchanged: 2^67 * k steps of the Weyl sequence are 0 mod 2^32.
    return st;
}

// ---------------------------------------------------------------------------------------
// Environment texture: PocaTextureUtils::GetTexture2D (textures.cu:68-71) over the cudaArray
// filled by AddTexByFile (textures.cu:14-62): uchar4, normalized coords, Mirror addressing,
// Linear filter, NormalizedFloat read.  Only `valid_cols` columns hold data (textures.cu:32-33
// copies width BYTES per row); the rest are read as 0 (UNPINNED: uninitialised in CUDA).
// Bilinear weights are quantised to 1/256 with round-to-nearest (CUDA guide: 9-bit fixed
// point, 8 fractional bits; rounding mode UNPINNED).
// ---------------------------------------------------------------------------------------
// Address modes (cudaTextureAddressMode values) and filter modes (cudaTextureFilterMode).
enum { ADDR_WRAP = 0, ADDR_CLAMP = 1, ADDR_MIRROR = 2, ADDR_BORDER = 3 };
enum { FILTER_POINT = 0, FILTER_LINEAR = 1 };

struct Env {
    const uint8_t* rgba;   // valid_cols x h, row pitch valid_cols*4
    int w, h, valid_cols;
    int addr = ADDR_MIRROR, filter = FILTER_LINEAR;   // the sky's: AddTexByFile defaults (textures.h:9-11)
};

inline int mirror_index(int i, int n) {
    int period = 2 * n;
    int m = i % period;
    if (m < 0) m += period;
    if (m >= n) m = period - 1 - m;
    return m;
}

// Texel index after addressing; -1 = outside (border colour 0).
inline int address(int i, int n, int mode) {
    switch (mode) {
        case ADDR_WRAP: { int m = i % n; return m < 0 ? m + n : m; }
        case ADDR_CLAMP: return i < 0 ? 0 : (i >= n ? n - 1 : i);
        case ADDR_BORDER: return (i < 0 || i >= n) ? -1 : i;
        default: return mirror_index(i, n);
    }
}

inline void texel(const Env& e, int i, int j, float out[3]) {
    int x = address(i, e.w, e.addr), y = address(j, e.h, e.addr);
    if (x < 0 || y < 0 || x >= e.valid_cols || e.rgba == nullptr) { out[0] = out[1] = out[2] = 0.0f; return; }
    const uint8_t* p = e.rgba + ((size_t)y * e.valid_cols + x) * 4;
    out[0] = (float)p[0] / 255.0f;
    out[1] = (float)p[1] / 255.0f;
    out[2] = (float)p[2] / 255.0f;
}

f3 tex2d(const Env& e, float u, float v) {
    if (e.filter == FILTER_POINT) {
        float x = u * (float)e.w, y = v * (float)e.h;
        if (!(x > -1e7f && x < 1e7f && y > -1e7f && y < 1e7f)) return mk1(0.0f);
        float t[3];
        texel(e, (int)floorf(x), (int)floorf(y), t);
        return mk(t[0], t[1], t[2]);
    }
    float x = u * (float)e.w - 0.5f;
    float y = v * (float)e.h - 0.5f;
    if (!(x > -1e7f && x < 1e7f && y > -1e7f && y < 1e7f)) return mk1(0.0f);  // NaN/huge guard
    float fx = floorf(x), fy = floorf(y);
    float a = floorf((x - fx) * 256.0f + 0.5f) * 0.00390625f;
    float b = floorf((y - fy) * 256.0f + 0.5f) * 0.00390625f;
    int i0 = (int)fx, j0 = (int)fy;
    float t00[3], t10[3], t01[3], t11[3];
    texel(e, i0, j0, t00);
    texel(e, i0 + 1, j0, t10);
    texel(e, i0, j0 + 1, t01);
    texel(e, i0 + 1, j0 + 1, t11);
    float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b), w01 = (1.0f - a) * b, w11 = a * b;
    float r[3];
    for (int c = 0; c < 3; ++c) r[c] = ((w00 * t00[c] + w10 * t10[c]) + w01 * t01[c]) + w11 * t11[c];
    return mk(r[0], r[1], r[2]);
}

// Material textures (§8(f) rank 4): handle -> texels, bound by or_bind_texture the way the
// app would keep the cudaTextureObject_t returned by AddTexByFile.
struct TexRec {
    std::vector<uint8_t> rgba;
    Env env;
};
std::mutex g_tex_mu;
std::vector<std::pair<uint64_t, TexRec*>> g_textures;

const TexRec* find_texture(uint64_t handle) {
    std::lock_guard<std::mutex> g(g_tex_mu);
    for (auto& t : g_textures) if (t.first == handle) return t.second;
    return nullptr;
}

// ---------------------------------------------------------------------------------------
// Scene BVH — SceneBVH::Divide / BuildBVHInCpu (bvh.cu:31-95), node = bvh.h:32-38.
// ---------------------------------------------------------------------------------------
struct Node {
    f3 bmin, bmax;
    bool is_object;
    int left, right;
    int obj;          // index into the object array (the reference stores a by-value copy)
};

f3 aabb_max(const Object& o) {                                  // object.cu:134-151
    float tol = BOUNCE_RAY_TMIN * 5.f;
    switch (o.type) {
        case PRIM_SPHERE: return add(o.center, mk1(ABS_(o.radius)));
        case PRIM_PLATFORM: return mk(DEFAULT_RAY_TMAX * 5, o.y_pos + tol, DEFAULT_RAY_TMAX * 5);
        case PRIM_CYLINDER:
            return mk(o.center.x + ABS_(o.radius), o.center.y + o.height / 2 + tol, o.center.z + ABS_(o.radius));
        default: return mk1(0.0f);   // reference: uninitialised
    }
}

f3 aabb_min(const Object& o) {                                  // object.cu:153-170
    float tol = BOUNCE_RAY_TMIN * 5.f;
    switch (o.type) {
        case PRIM_SPHERE: return sub(o.center, mk1(ABS_(o.radius)));
        case PRIM_PLATFORM: return mk(-DEFAULT_RAY_TMAX * 5, o.y_pos - tol, -DEFAULT_RAY_TMAX * 5);
        case PRIM_CYLINDER:
            return mk(o.center.x - ABS_(o.radius), o.center.y - o.height / 2 - tol, o.center.z - ABS_(o.radius));
        default: return mk1(0.0f);
    }
}

struct Bvh {
    std::vector<Node> nodes;
    const Object* objs;
    // diagnostic ordered walk only (trace_ray_ordered):
    std::vector<int> axis;       // split axis per internal node
    std::vector<int> rank;       // right-first preorder position
    struct WNode { f3 bmin, bmax; int left, right, obj, axis; };
    std::vector<WNode> walk;     // binned-SAH tree over the bounded primitives
    int walk_root = -1;
    std::vector<int> unbounded;  // platform leaves of `walk`, by rank
    std::vector<int> rank_of_obj;
};

// std::sort in the reference (bvh.cu:67-80) is unstable; ties between equal centroids are
// implementation-defined.  The restatement uses stable_sort (documented tie rule; the test
// scenes have no centroid ties).
int divide(Bvh& bvh, std::vector<int>& idx, int l, int r) {      // bvh.cu:31-90
    if (l >= r) return -1;
    int ret = (int)bvh.nodes.size();
    bvh.nodes.push_back(Node{});
    const Object* O = bvh.objs;
    f3 lmin = aabb_min(O[idx[l]]), lmax = aabb_max(O[idx[l]]);
    if (l == r - 1) {
        Node& n = bvh.nodes[ret];
        n.left = n.right = -1;
        n.bmin = lmin; n.bmax = lmax;
        n.is_object = true;
        n.obj = idx[l];
        return ret;
    }
    float minx = lmin.x, miny = lmin.y, minz = lmin.z;
    float maxx = lmax.x, maxy = lmax.y, maxz = lmax.z;
    for (int i = l + 1; i < r; ++i) {
        f3 cmin = aabb_min(O[idx[i]]), cmax = aabb_max(O[idx[i]]);
        minx = MIN_(minx, cmin.x); miny = MIN_(miny, cmin.y); minz = MIN_(minz, cmin.z);
        maxx = MAX_(maxx, cmax.x); maxy = MAX_(maxy, cmax.y); maxz = MAX_(maxz, cmax.z);
    }
    float span_x = maxx - minx, span_y = maxy - miny, span_z = maxz - minz;
    int axis = (span_x >= span_y && span_x >= span_z) ? 0 : (span_y >= span_z ? 1 : 2);
    auto centroid = [&](int k) {
        f3 a = aabb_min(O[k]), b = aabb_max(O[k]);
        float lo = axis == 0 ? a.x : axis == 1 ? a.y : a.z;
        float hi = axis == 0 ? b.x : axis == 1 ? b.y : b.z;
        return (lo + hi) / 2;
    };
    std::stable_sort(idx.begin() + l, idx.begin() + r, [&](int a, int b) { return centroid(a) < centroid(b); });
    int mid = (l + r) / 2;
    if ((int)bvh.axis.size() <= ret) bvh.axis.resize(ret + 1, 0);
    bvh.axis[ret] = axis;
    int left = divide(bvh, idx, l, mid);
    int right = divide(bvh, idx, mid, r);
    Node& n = bvh.nodes[ret];
    n.left = left; n.right = right;
    n.bmin = mk(minx, miny, minz);
    n.bmax = mk(maxx, maxy, maxz);
    n.is_object = false;
    n.obj = -1;
    return ret;
}

void build_walk_tree(Bvh& bvh);

void build_bvh(Bvh& bvh, const Object* objs, int n) {
    bvh.objs = objs;
    bvh.nodes.clear();
    std::vector<int> idx(n);
    for (int i = 0; i < n; ++i) idx[i] = i;
    divide(bvh, idx, 0, n);
    bvh.axis.resize(bvh.nodes.size(), 0);
    bvh.rank.assign(bvh.nodes.size(), 0);
    int pos = 0;
    std::vector<int> st;
    if (n > 0) st.push_back(0);
    while (!st.empty()) {                 // the reference's pop order: right child first
        int ni = st.back();
        st.pop_back();
        bvh.rank[ni] = pos++;
        if (!bvh.nodes[ni].is_object) { st.push_back(bvh.nodes[ni].left); st.push_back(bvh.nodes[ni].right); }
    }
    build_walk_tree(bvh);
}

// Walk tree of the diagnostic ordered walk: platforms (unbounded) are tested first; the other
// primitives get a binned-SAH tree (16 bins per axis, one primitive per leaf), built with the
// same float operations as libcpt's host builder (cpt_capi.cpp, namespace sah).
namespace walk_sah {
constexpr int NB = 16;
inline float comp(f3 v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }
inline f3 fmin3(f3 a, f3 b) { return mk(MIN_(a.x, b.x), MIN_(a.y, b.y), MIN_(a.z, b.z)); }
inline f3 fmax3(f3 a, f3 b) { return mk(MAX_(a.x, b.x), MAX_(a.y, b.y), MAX_(a.z, b.z)); }
inline float area(f3 lo, f3 hi) {
    float dx = hi.x - lo.x, dy = hi.y - lo.y, dz = hi.z - lo.z;
    return 2.f * (dx * dy + dy * dz + dz * dx);
}
inline int bin_of(float c, float e0, float e1) { return std::min(NB - 1, (int)((c - e0) / (e1 - e0) * NB)); }

int leaf(Bvh& b, int o) {
    Bvh::WNode n;
    n.bmin = aabb_min(b.objs[o]);
    n.bmax = aabb_max(b.objs[o]);
    n.left = n.right = -1;
    n.obj = o;
    n.axis = 0;
    b.walk.push_back(n);
    return (int)b.walk.size() - 1;
}

int build(Bvh& b, std::vector<int>& idx, int l, int r) {
    const Object* O = b.objs;
    if (r - l == 1) return leaf(b, idx[l]);
    f3 lo = aabb_min(O[idx[l]]), hi = aabb_max(O[idx[l]]);
    f3 clo = mk(1e30f, 1e30f, 1e30f), chi = mk(-1e30f, -1e30f, -1e30f);
    std::vector<float> cen(3 * (r - l));
    for (int i = l; i < r; ++i) {
        f3 a = aabb_min(O[idx[i]]), c2 = aabb_max(O[idx[i]]);
        lo = fmin3(lo, a);
        hi = fmax3(hi, c2);
        f3 c = mk((a.x + c2.x) * .5f, (a.y + c2.y) * .5f, (a.z + c2.z) * .5f);
        cen[3 * (i - l)] = c.x; cen[3 * (i - l) + 1] = c.y; cen[3 * (i - l) + 2] = c.z;
        clo = fmin3(clo, c);
        chi = fmax3(chi, c);
    }
    float best = 3.0e38f;
    int best_axis = -1, best_bin = -1;
    for (int axis = 0; axis < 3; ++axis) {
        float e0 = comp(clo, axis), e1 = comp(chi, axis);
        if (!(e1 > e0)) continue;
        int cnt[NB] = {0};
        f3 blo[NB], bhi[NB];
        for (int k = 0; k < NB; ++k) { blo[k] = mk(1e30f, 1e30f, 1e30f); bhi[k] = mk(-1e30f, -1e30f, -1e30f); }
        for (int i = l; i < r; ++i) {
            int k = bin_of(cen[3 * (i - l) + axis], e0, e1);
            cnt[k]++;
            blo[k] = fmin3(blo[k], aabb_min(O[idx[i]]));
            bhi[k] = fmax3(bhi[k], aabb_max(O[idx[i]]));
        }
        for (int sp = 1; sp < NB; ++sp) {
            int nl = 0, nr = 0;
            f3 llo = mk(1e30f, 1e30f, 1e30f), lhi = mk(-1e30f, -1e30f, -1e30f), rlo = llo, rhi = lhi;
            for (int k = 0; k < sp; ++k) if (cnt[k]) { nl += cnt[k]; llo = fmin3(llo, blo[k]); lhi = fmax3(lhi, bhi[k]); }
            for (int k = sp; k < NB; ++k) if (cnt[k]) { nr += cnt[k]; rlo = fmin3(rlo, blo[k]); rhi = fmax3(rhi, bhi[k]); }
            if (!nl || !nr) continue;
            float cost = area(llo, lhi) * nl + area(rlo, rhi) * nr;
            if (cost < best) { best = cost; best_axis = axis; best_bin = sp; }
        }
    }
    int axis, mid;
    if (best_axis < 0) {
        axis = 0;
        mid = (l + r) / 2;
    } else {
        axis = best_axis;
        float e0 = comp(clo, axis), e1 = comp(chi, axis);
        std::vector<int> lhs, rhs;
        for (int i = l; i < r; ++i) (bin_of(cen[3 * (i - l) + axis], e0, e1) < best_bin ? lhs : rhs).push_back(idx[i]);
        std::copy(lhs.begin(), lhs.end(), idx.begin() + l);
        std::copy(rhs.begin(), rhs.end(), idx.begin() + l + (int)lhs.size());
        mid = l + (int)lhs.size();
    }
    int me = (int)b.walk.size();
    b.walk.push_back(Bvh::WNode{});
    int L = build(b, idx, l, mid), R = build(b, idx, mid, r);
    Bvh::WNode& n = b.walk[me];
    n.bmin = lo; n.bmax = hi;
    n.left = L; n.right = R; n.obj = -1; n.axis = axis;
    return me;
}
}  // namespace walk_sah

void build_walk_tree(Bvh& bvh) {
    const int n_obj = (int)(bvh.nodes.empty() ? 0 : (bvh.nodes.size() + 1) / 2);
    bvh.walk.clear();
    bvh.unbounded.clear();
    bvh.walk_root = -1;
    bvh.rank_of_obj.assign(n_obj, 0);
    for (size_t i = 0; i < bvh.nodes.size(); ++i)
        if (bvh.nodes[i].is_object) bvh.rank_of_obj[bvh.nodes[i].obj] = bvh.rank[i];
    std::vector<std::pair<int, int>> flat;
    std::vector<int> idx;
    for (int o = 0; o < n_obj; ++o) {
        if (bvh.objs[o].type == PRIM_PLATFORM) flat.emplace_back(bvh.rank_of_obj[o], o);
        else idx.push_back(o);
    }
    std::sort(flat.begin(), flat.end());
    for (auto& f : flat) bvh.unbounded.push_back(walk_sah::leaf(bvh, f.second));
    if (!idx.empty()) bvh.walk_root = walk_sah::build(bvh, idx, 0, (int)idx.size());
}

// ---------------------------------------------------------------------------------------
// Ray / intersection (ray_tracing_common.h:14-35, object.cu:10-128)
// ---------------------------------------------------------------------------------------
struct Ray { f3 origin, dir; float tmin, tmax; };
struct Attr { f3 normal, hit_pos; };

bool sphere_test(const Object& s, Ray& ray, Attr& attr) {        // object.cu:10-35
    f3 A_C = sub(ray.origin, s.center);
    f3 B = ray.dir;
    float a = dot(B, B);
    float b = dot(A_C, B);
    float c = dot(A_C, A_C) - s.radius * s.radius;
    float disc = b * b - a * c;
    if (disc > 0) {
        float temp = (-b - sqrtf(disc)) / a;
        if (temp < ray.tmax && temp > ray.tmin) {
            ray.tmax = temp;
            attr.hit_pos = add(ray.origin, mul(temp, ray.dir));
            f3 normal = sub(attr.hit_pos, s.center);
            attr.normal = divs(normal, s.radius);
            return true;
        }
        temp = (-b + sqrtf(disc)) / a;
        if (temp < ray.tmax && temp > ray.tmin) {
            ray.tmax = temp;
            attr.hit_pos = add(ray.origin, mul(temp, ray.dir));
            attr.normal = normalize(sub(attr.hit_pos, s.center));
            return true;
        }
    }
    return false;
}

bool platform_test(const Object& p, Ray& ray, Attr& attr) {      // object.cu:37-48
    if ((ray.origin.y < p.y_pos && ray.dir.y > 0.f) || (ray.origin.y > p.y_pos && ray.dir.y < 0.f)) {
        float temp = (p.y_pos - ray.origin.y) / ray.dir.y;
        if (temp < ray.tmax && temp > ray.tmin) {
            ray.tmax = temp;
            attr.hit_pos = add(ray.origin, mul(temp, ray.dir));
            attr.normal = normalize(mk(0, -ray.dir.y, 0));
            return true;
        }
    }
    return false;
}

bool cap_test(const Object& cy, Ray& ray, Attr& attr, float ypos) {  // object.cu:52-77 (one cap)
    if ((ray.origin.y < ypos && ray.dir.y > 0.f) || (ray.origin.y > ypos && ray.dir.y < 0.f)) {
        float temp = (ypos - ray.origin.y) / ray.dir.y;
        f3 hit_pos = add(ray.origin, mul(temp, ray.dir));
        if (temp < ray.tmax && temp > ray.tmin &&
            sqrtf((hit_pos.x - cy.center.x) * (hit_pos.x - cy.center.x) +
                  (hit_pos.z - cy.center.z) * (hit_pos.z - cy.center.z)) < cy.radius) {
            ray.tmax = temp;
            attr.hit_pos = hit_pos;
            attr.normal = normalize(mk(0, -ray.dir.y, 0));
            return true;
        }
    }
    return false;
}

bool cylinder_test(const Object& cy, Ray& ray, Attr& attr) {     // object.cu:50-112
    bool ret = false;
    float upper = cy.center.y + cy.height / 2;
    if (cap_test(cy, ray, attr, upper)) ret = true;
    float lower = cy.center.y - cy.height / 2;
    if (cap_test(cy, ray, attr, lower)) ret = true;
    float dx = ray.dir.x, dz = ray.dir.z, r = cy.radius;
    float cx = ray.origin.x - cy.center.x;
    float cz = ray.origin.z - cy.center.z;
    float a = dx * dx + dz * dz;
    float b = cx * dx + cz * dz;
    float c = cx * cx + cz * cz - r * r;
    float disc = b * b - a * c;
    if (disc > 0.f) {
        float temp = (-b - sqrtf(disc)) / a;
        f3 hit_pos = add(ray.origin, mul(temp, ray.dir));
        if (temp < ray.tmax && temp > ray.tmin && hit_pos.y > lower && hit_pos.y < upper) {
            ray.tmax = temp;
            attr.hit_pos = hit_pos;
            attr.normal = normalize(mk(hit_pos.x - cy.center.x, 0.f, hit_pos.z - cy.center.z));
            ret = true;
        }
        temp = (-b + sqrtf(disc)) / a;
        hit_pos = add(ray.origin, mul(temp, ray.dir));
        if (temp < ray.tmax && temp > ray.tmin && hit_pos.y > lower && hit_pos.y < upper) {
            ray.tmax = temp;
            attr.hit_pos = hit_pos;
            attr.normal = normalize(mk(hit_pos.x - cy.center.x, 0.f, hit_pos.z - cy.center.z));
            ret = true;
        }
    }
    return ret;
}

bool intersection_test(const Object& o, Ray& ray, Attr& attr) {  // object.cu:114-128
    switch (o.type) {
        case PRIM_SPHERE: return sphere_test(o, ray, attr);
        case PRIM_PLATFORM: return platform_test(o, ray, attr);
        case PRIM_CYLINDER: return cylinder_test(o, ray, attr);
        default: return false;
    }
}

struct Stats { uint64_t segments, nodes, prims, hits, misses, fallbacks; };

// SceneBVH::TraceRay (bvh.cu:167-205): DFS, explicit stack, leaf test before slab test,
// left pushed before right (right popped first), ray taken BY VALUE.
bool slab_pass(const Node& n, const Ray& ray);
bool trace_ray_ordered(const Bvh& bvh, Ray ray, Attr& attr, int& hit_obj, Stats& st);
static int g_walk_ordered = 0;
static std::atomic<uint64_t> g_last_fallbacks{0};   // diagnostic walk: certificate fallbacks of the last render
// Diagnostic hook for walk experiments compiled against this file (never set by the library).
static bool (*g_trace_hook)(const Bvh&, Ray, Attr&, int&, Stats&) = nullptr;

bool trace_ray_ref(const Bvh& bvh, Ray ray, Attr& attr, int& hit_obj, Stats& st);

bool trace_ray(const Bvh& bvh, Ray ray, Attr& attr, int& hit_obj, Stats& st) {
    if (bvh.nodes.empty()) return false;
    if (g_trace_hook) return g_trace_hook(bvh, ray, attr, hit_obj, st);
    if (g_walk_ordered) return trace_ray_ordered(bvh, ray, attr, hit_obj, st);
    return trace_ray_ref(bvh, ray, attr, hit_obj, st);
}

bool trace_ray_ref(const Bvh& bvh, Ray ray, Attr& attr, int& hit_obj, Stats& st) {
    int stack[512];
    int top = 0;
    stack[top++] = 0;
    bool ret = false;
    while (top > 0) {
        int ni = stack[--top];
        if (ni == -1) continue;
        const Node& n = bvh.nodes[ni];
        st.nodes++;
        if (n.is_object) {
            st.prims++;
            if (intersection_test(bvh.objs[n.obj], ray, attr)) { hit_obj = n.obj; ret = true; }
        }
        float local_tmin = -DEFAULT_RAY_TMAX * 2, local_tmax = DEFAULT_RAY_TMAX * 2;
        if (ray.dir.x != 0.f) {
            float t0 = (n.bmin.x - ray.origin.x) / ray.dir.x;
            float t1 = (n.bmax.x - ray.origin.x) / ray.dir.x;
            local_tmin = MAX_(local_tmin, MIN_(t0, t1));
            local_tmax = MIN_(local_tmax, MAX_(t0, t1));
        }
        if (ray.dir.y != 0.f) {
            float t0 = (n.bmin.y - ray.origin.y) / ray.dir.y;
            float t1 = (n.bmax.y - ray.origin.y) / ray.dir.y;
            local_tmin = MAX_(local_tmin, MIN_(t0, t1));
            local_tmax = MIN_(local_tmax, MAX_(t0, t1));
        }
        if (ray.dir.z != 0.f) {
            float t0 = (n.bmin.z - ray.origin.z) / ray.dir.z;
            float t1 = (n.bmax.z - ray.origin.z) / ray.dir.z;
            local_tmin = MAX_(local_tmin, MIN_(t0, t1));
            local_tmax = MIN_(local_tmax, MAX_(t0, t1));
        }
        if (local_tmin > local_tmax || local_tmin > ray.tmax || local_tmax < ray.tmin) continue;
        if (top + 2 > 512) return ret;   // reference would overflow; unreachable for sane trees
        stack[top++] = n.left;
        stack[top++] = n.right;
    }
    return ret;
}

// ---------------------------------------------------------------------------------------
// DIAGNOSTIC ONLY (or_set_walk(1)); not the reference algorithm.  A restatement of this
// build's CPT_TRAVERSAL_ORDERED walk, used by tests/tools to compare the ordered walk's own
// node/primitive counts and to study where it can part from the reference.  The unbounded
// (platform) leaves are tested first, then the walk tree (bvh.walk) is walked with the child
// nearer along the split axis (by the ray's direction sign) first.  A leaf the reference
// meets earlier than the current closest primitive (lower right-first preorder rank) is
// tested against next_up(tmax), i.e. wins ties.
// ---------------------------------------------------------------------------------------
bool slab_pass(const Node& n, const Ray& ray) {                 // bvh.cu:181-200
    float local_tmin = -DEFAULT_RAY_TMAX * 2, local_tmax = DEFAULT_RAY_TMAX * 2;
    const float o[3] = {ray.origin.x, ray.origin.y, ray.origin.z}, d[3] = {ray.dir.x, ray.dir.y, ray.dir.z};
    const float lo[3] = {n.bmin.x, n.bmin.y, n.bmin.z}, hi[3] = {n.bmax.x, n.bmax.y, n.bmax.z};
    for (int a = 0; a < 3; ++a) {
        if (d[a] == 0.f) continue;
        float t0 = (lo[a] - o[a]) / d[a], t1 = (hi[a] - o[a]) / d[a];
        local_tmin = MAX_(local_tmin, MIN_(t0, t1));
        local_tmax = MIN_(local_tmax, MAX_(t0, t1));
    }
    return !(local_tmin > local_tmax || local_tmin > ray.tmax || local_tmax < ray.tmin);
}

// The product's conservative slab (cpt_path.hpp slab_reject<FAST, true>, slab_pass, RayK): f32
// reciprocals i = 1/d, scaled to in = i (1 - 1e-3) for entry planes and if = i (1 + 1e-3) for
// exit planes; a plane p is entered at fma(p, in, cn) and left at fma(p, if, cf), with
// cn = -(o in) - 2^-20 |o in| and cf = (-(o if) + 2^-20 |o if|) + SLAB_ABS (the entry plane is
// the min plane when i >= 0); skipped axes for |d| < 1e-30 (i = 0, c = -+2e30).  The box
// passes iff max(lo, t3') <= min(hi, limit'), t3' = t3 - 1e-3 |t3| with
// t3 = (tmin - 1e-4) * 1.002, limit' = ((tmax + 1e-4) * 1.002) * 1.001.
bool slab_pass_conservative(const Bvh::WNode& n, const Ray& ray) {
    const float BIG = DEFAULT_RAY_TMAX * 2;
    const float REL = 1e-3f, ABS = 1e-4f, SHRINK = 1.0f - REL, GROW = 1.0f + REL;
    const float SLAB_ABS = 2.0f * ABS * (1.0f + 2.0f * REL) * GROW + 1e-6f;
    const float o[3] = {ray.origin.x, ray.origin.y, ray.origin.z}, d[3] = {ray.dir.x, ray.dir.y, ray.dir.z};
    const float a[3] = {n.bmin.x, n.bmin.y, n.bmin.z}, b[3] = {n.bmax.x, n.bmax.y, n.bmax.z};
    float l[3], h[3];
    for (int k = 0; k < 3; ++k) {
        const float inv = fabsf(d[k]) >= 1e-30f ? 1.0f / d[k] : 0.0f;
        const float in = inv * SHRINK, ig = inv * GROW;
        const float pn = o[k] * in, pf = o[k] * ig;
        const float cn = inv != 0.0f ? -pn - fabsf(pn) * 0x1p-20f : -BIG;
        const float cf = inv != 0.0f ? (-pf + fabsf(pf) * 0x1p-20f) + SLAB_ABS : BIG;
        const bool pos = in >= 0.0f;
        l[k] = fmaf(pos ? a[k] : b[k], in, cn);
        h[k] = fmaf(pos ? b[k] : a[k], ig, cf);
    }
    const float tlim = ((ray.tmax + ABS) * (1.0f + 2.0f * REL)) * GROW;
    const float t3r = (ray.tmin - 1e-4f) * (1.0f + 2e-3f);
    const float t3 = t3r - REL * fabsf(t3r);
    const float lo = fmaxf(fmaxf(fmaxf(l[0], l[1]), l[2]), t3);
    const float hi = fminf(fminf(h[0], h[1]), h[2]);
    return lo <= fminf(hi, tlim);
}

bool trace_ray_ordered(const Bvh& bvh, Ray ray, Attr& attr, int& hit_obj, Stats& st) {
    const Ray ray0 = ray;   // TraceRay's by-value ray, for the fallback
    bool ret = false;
    int best_rank = 0x7fffffff, win = -1;
    auto leaf = [&](int wi) {
        const int o = bvh.walk[wi].obj;
        st.nodes++;
        st.prims++;
        Ray r2 = ray;
        if (bvh.rank_of_obj[o] < best_rank) {
            uint32_t u;
            std::memcpy(&u, &r2.tmax, 4);
            u += 1;
            std::memcpy(&r2.tmax, &u, 4);
        }
        if (intersection_test(bvh.objs[o], r2, attr)) {
            ray.tmax = r2.tmax;
            hit_obj = o;
            win = o;
            best_rank = bvh.rank_of_obj[o];
            ret = true;
        }
    };
    for (int wi : bvh.unbounded) leaf(wi);
    if (bvh.walk_root >= 0) {
        int stack[512];
        int top = 0;
        stack[top++] = bvh.walk_root;
        const float d[3] = {ray.dir.x, ray.dir.y, ray.dir.z};
        while (top > 0) {
            int wi = stack[--top];
            const Bvh::WNode& n = bvh.walk[wi];
            if (n.obj >= 0) { leaf(wi); continue; }
            st.nodes++;
            if (!slab_pass_conservative(n, ray)) continue;
            if (top + 2 > 512) break;
            const bool right_first = d[n.axis] < 0.f;
            stack[top++] = right_first ? n.left : n.right;
            stack[top++] = right_first ? n.right : n.left;
        }
    }
    if (win >= 0) {
        // certificate: the winner's own box passes the exact slab test at tmax = t_win
        Node box;
        box.bmin = aabb_min(bvh.objs[win]);
        box.bmax = aabb_max(bvh.objs[win]);
        if (!slab_pass(box, ray)) {
            st.fallbacks++;
            return trace_ray_ref(bvh, ray0, attr, hit_obj, st);
        }
    }
    return ret;
}

// ---------------------------------------------------------------------------------------
// Shading (material.cu).  Payload mirrors RayPayload (ray_tracing_common.h:21-30).
// ---------------------------------------------------------------------------------------
struct Payload {
    Ray ray;
    f3 radiance, attenuation, hit_pos, bounce_dir;
    uint32_t depth;
};

// to_world (ray_tracing_math.hpp:51-63)
f3 to_world(f3 a, f3 N) {
    f3 B, C;
    if (fabsf(N.x) > fabsf(N.y)) {
        float invLen = 1.0f / sqrtf(N.x * N.x + N.z * N.z);
        C = mk(N.z * invLen, 0.0f, -N.x * invLen);
    } else {
        float invLen = 1.0f / sqrtf(N.y * N.y + N.z * N.z);
        C = mk(0.f, N.z * invLen, -N.y * invLen);
    }
    B = cross(C, N);
    return add(add(mul(a.x, B), mul(a.y, C)), mul(a.z, N));
}

// schlick (ray_tracing_math.hpp:65-69).  pow(float, int) resolves to CUDA's float overload
// in device code (UNPINNED: ISO C++ would promote to double).
float schlick(float cosine, float ref_idx) {
    float r0 = (1 - ref_idx) / (1 + ref_idx);
    r0 *= r0;
    return r0 + (1 - r0) * dm_pow5f(1 - cosine);
}

// refract (ray_tracing_math.hpp:71-80): discriminant in double (1.0 literal), stored float.
bool refract(f3 v, f3 n, float ni_over_nt, f3& refracted) {
    f3 uv = normalize(v);
    float dt = dot(uv, n);
    float discriminant = (float)(1.0 - (double)(ni_over_nt * ni_over_nt * (1 - dt * dt)));
    if (discriminant > 0) {
        refracted = normalize(sub(mul(ni_over_nt, sub(uv, mul(n, dt))), mul(n, sqrtf(discriminant))));
        return true;
    }
    return false;
}

// Shared lobe: z = pow(x1, 1/alpha) (double pow), r = sqrtf(1 - z^2), phi = 2*M_PI*x2 (double).
inline f3 lobe(float x_1, float x_2, double inv_alpha) {
    float z = (float)dm_pow((double)x_1, inv_alpha);
    float r = sqrtf(1.0f - z * z);
    float phi = (float)(2 * REF_PI * (double)x_2);
    return mk(r * dm_cosf(phi), r * dm_sinf(phi), z);
}

// Material::GetKd (material.cu:11-18), always called with (x, y) = (0, 0): the texture's
// sample at normalized (0, 0) for a textured material (an unbound handle reads 0), else kd_.
// Emission keeps reading kd_, which aliases tex_ in a textured material (material.cu:36).
f3 get_kd(const Material& m) {
    if (!m.have_tex) return m.u.kd;
    const TexRec* t = find_texture(m.u.tex);
    return t ? tex2d(t->env, 0.0f, 0.0f) : mk1(0.0f);
}

void diffuse_shader(const Material& m, Payload& p, f3 position, f3 normal, f3 in_ray_dir, Xorwow& rng) {  // :20-38
    (void)in_ray_dir;
    float x_1 = uniform(rng), x_2 = uniform(rng);
    f3 localRay = lobe(x_1, x_2, 1.0 / 2);
    p.bounce_dir = to_world(localRay, normal);
    float cosalpha = dot(normal, p.bounce_dir);
    p.attenuation = cosalpha > 0.0f ? get_kd(m) : mk(0.0f, 0.0f, 0.0f);
    p.radiance = mul(m.emit_intensity, m.u.kd);
    p.hit_pos = position;
}

void mirror_shader(const Material& m, Payload& p, f3 position, f3 normal, f3 in_ray_dir, Xorwow& rng) {  // :40-64
    float s = m.smoothness;
    float alpha = dm_powf(1000.0f, s);
    float x_1 = uniform(rng), x_2 = uniform(rng);
    f3 localRay = lobe(x_1, x_2, 1.0 / (double)alpha);
    f3 reflect_dir = reflect(in_ray_dir, normal);
    f3 wo = to_world(localRay, reflect_dir);
    float cosalpha = dot(normal, wo);
    p.attenuation = cosalpha > 0.0f ? get_kd(m) : mk(0.0f, 0.0f, 0.0f);
    p.bounce_dir = wo;
    p.radiance = mul(m.emit_intensity, m.u.kd);
    p.hit_pos = position;
}

void metal_shader(const Material& m, Payload& p, f3 position, f3 normal, f3 in_ray_dir, Xorwow& rng) {  // :66-99
    float x_1 = uniform(rng), x_2 = uniform(rng);
    float s = m.smoothness;
    float alpha = dm_powf(1000.0f, s);
    float reflectivity = m.reflectivity;
    if (uniform(rng) < reflectivity) {
        f3 localRay = lobe(x_1, x_2, 1.0 / (double)alpha);
        p.bounce_dir = to_world(localRay, reflect(in_ray_dir, normal));
    } else {
        f3 localRay = lobe(x_1, x_2, 1.0 / 2.0);
        p.bounce_dir = to_world(localRay, normal);
    }
    p.attenuation = dot(p.bounce_dir, normal) < 0 ? mk(0.0f, 0.0f, 0.0f) : get_kd(m);
    p.radiance = mul(m.emit_intensity, m.u.kd);
    p.hit_pos = position;
}

void glass_shader(const Material& m, Payload& p, f3 position, f3 normal, f3 in_ray_dir, Xorwow& rng) {  // :101-143
    float x_1 = uniform(rng), x_2 = uniform(rng);
    float alpha = dm_powf(1000.0f, m.smoothness);
    f3 localRay = lobe(x_1, x_2, 1.0 / (double)alpha);
    f3 outward_normal, refracted = mk1(0.0f);
    float ni_over_nt, reflect_prob, cosine;
    in_ray_dir = normalize(in_ray_dir);
    if (dot(in_ray_dir, normal) > 0) {
        outward_normal = neg(normal);
        ni_over_nt = m.refractive_index;
        cosine = dot(in_ray_dir, normal);
        cosine = sqrtf(1 - m.refractive_index * m.refractive_index * (1 - cosine * cosine));
    } else {
        outward_normal = normal;
        ni_over_nt = 1.f / m.refractive_index;
        cosine = -dot(in_ray_dir, normal);
    }
    if (refract(in_ray_dir, outward_normal, ni_over_nt, refracted)) reflect_prob = schlick(cosine, m.refractive_index);
    else reflect_prob = 1.0f;
    if (uniform(rng) < reflect_prob) p.bounce_dir = to_world(localRay, reflect(in_ray_dir, normal));
    else p.bounce_dir = to_world(localRay, refracted);
    p.attenuation = get_kd(m);
    p.radiance = mul(m.emit_intensity, m.u.kd);
    p.hit_pos = position;
}

// Material::EvalAttenuationAndCreateRay (material.cu:145-163) — note the Metal/Mirror swap.
void eval_material(const Material& m, Payload& p, f3 position, f3 normal, f3 in_ray_dir, Xorwow& rng) {
    switch (m.type) {
        case MAT_DIFFUSE: diffuse_shader(m, p, position, normal, in_ray_dir, rng); break;
        case MAT_METAL: mirror_shader(m, p, position, normal, in_ray_dir, rng); break;
        case MAT_MIRROR: metal_shader(m, p, position, normal, in_ray_dir, rng); break;
        case MAT_GLASS: glass_shader(m, p, position, normal, in_ray_dir, rng); break;
        default: diffuse_shader(m, p, position, normal, in_ray_dir, rng);
    }
}

// Miss (path_tracer.cu:117-122)
void miss(const Env& env, Payload& p) {
    f3 d = normalize(p.ray.dir);
    float v = (float)((double)dm_asinf(d.z) / REF_PI + 0.5);
    float u = (float)((double)(dm_atanf(d.y / d.x) / 2) / REF_PI);
    p.radiance = tex2d(env, u, v);
    p.depth = MAX_RECURSION_DEPTH_SET;
}

// MotionalCamera::RayGen (motional_camera.cu:202-213); the three draws are taken left to
// right (argument evaluation order of make_float3 is unspecified; nvcc evaluates L->R).
Ray ray_gen(const Camera& c, int x, int y, Xorwow& rng) {
    float r1 = uniform(rng), r2 = uniform(rng), r3 = uniform(rng);
    f3 rd = mul(c.lens_radius, mk(r1, r2, r3));
    f3 offset = add(mul(c.u, rd.x), mul(c.v, rd.y));
    float dx = float(x) / float(c.width);
    float dy = float(y) / float(c.height);
    Ray ray;
    ray.origin = add(c.origin, offset);
    ray.dir = normalize(sub(sub(add(add(c.top_left, mul(dx, c.horizontal)), mul(dy, c.vertical)), c.origin), offset));
    ray.tmin = 0.f;
    ray.tmax = DEFAULT_RAY_TMAX;
    return ray;
}

struct PassOut { f3 radiance, normal; float depth; };

// SamplePixel body (path_tracer.cu:124-175) for one pixel and one pass.
PassOut sample_pixel(const Bvh& bvh, const Env& env, const Camera& cam, uint32_t max_depth, int x, int y,
                     Xorwow& rng, Stats& st) {
    f3 radiance = mk1(0.f), normals = mk1(0.f);
    float depth = 0.0f;
    Payload p;
    std::memset(&p, 0, sizeof(p));
    p.ray = ray_gen(cam, x, y, rng);
    f3 attenuation = mk1(1.f);
    p.depth = 0;
    bool first = false;
    while (p.depth < max_depth) {
        Attr attr;
        std::memset(&attr, 0, sizeof(attr));
        int hit_obj = -1;
        st.segments++;
        bool ret = trace_ray(bvh, p.ray, attr, hit_obj, st);
        if (ret) {
            st.hits++;
            // Object::ClosetHit (object.cu:130-132)
            eval_material(bvh.objs[hit_obj].material, p, attr.hit_pos, attr.normal, p.ray.dir, rng);
        } else {
            st.misses++;
            attr.hit_pos = add(p.ray.origin, mul(DEFAULT_RAY_TMAX, p.ray.dir));
            attr.normal = neg(p.ray.dir);
            miss(env, p);
        }
        radiance = add(radiance, mul(attenuation, p.radiance));
        attenuation = mul(attenuation, p.attenuation);
        if (!first) {
            normals = add(normals, attr.normal);
            depth += p.ray.tmax;
            first = true;
        }
        p.ray.origin = p.hit_pos;
        p.ray.dir = normalize(p.bounce_dir);
        p.ray.tmin = BOUNCE_RAY_TMIN;
        p.ray.tmax = DEFAULT_RAY_TMAX;
        p.depth++;
    }
    return PassOut{radiance, normals, depth};
}

struct RenderJob {
    const Bvh* bvh;
    Env env;
    Camera cam;
    const int32_t* rows;
    int n_rows;
    int spp;
    uint32_t max_depth;
    uint32_t* rng;      // planar [6][npix]
    float* accum;       // [npix][4]
    float* normal;      // [npix][3] or null
    float* depthbuf;    // [npix] or null
    int accumulate;
};

// DIAGNOSTIC (or_set_pixel_segments): per-pixel path segments of the next renders, i.e. the
// length of each pixel's sequential chain (tools/chain_costs.py).
uint32_t* g_pixel_segments = nullptr;
// DIAGNOSTIC (or_set_pass_trace): per pixel and pass, the RNG draws and path segments of the
// pass ([n_rows * W][spp] bytes each; tools/pass_trace.py).
uint8_t* g_pass_draws = nullptr;
uint8_t* g_pass_segs = nullptr;

void render_rows(const RenderJob& J, int thread, int nthreads, Stats& st) {
    const int W = J.cam.width;
    const size_t npix = (size_t)J.n_rows * W;
    for (int ri = thread; ri < J.n_rows; ri += nthreads) {
        int y = J.rows[ri];
        for (int x = 0; x < W; ++x) {
            size_t pix = (size_t)ri * W + x;
            Xorwow s;
            for (int k = 0; k < 5; ++k) s.v[k] = J.rng[k * npix + pix];
            s.d = J.rng[5 * npix + pix];
            float* a = J.accum + pix * 4;
            f3 sum = J.accumulate ? mk(a[0], a[1], a[2]) : mk1(0.0f);
            float cnt = J.accumulate ? a[3] : 0.0f;
            PassOut last{};
            const uint64_t seg0 = st.segments;
            for (int sidx = 0; sidx < J.spp; ++sidx) {
                const uint32_t d0 = s.d;
                const uint64_t sg0 = st.segments;
                last = sample_pixel(*J.bvh, J.env, J.cam, J.max_depth, x, y, s, st);
                if (g_pass_draws) {
                    // draws = (d1 - d0) / 362437 mod 2^32 (each draw adds the odd Weyl constant)
                    uint32_t inv = 362437u;
                    for (int i = 0; i < 5; ++i) inv *= 2u - 362437u * inv;
                    g_pass_draws[pix * J.spp + sidx] = (uint8_t)((s.d - d0) * inv);
                    g_pass_segs[pix * J.spp + sidx] = (uint8_t)(st.segments - sg0);
                }
                sum = add(sum, last.radiance);
                cnt += 1.0f;
            }
            a[0] = sum.x; a[1] = sum.y; a[2] = sum.z; a[3] = cnt;
            if (g_pixel_segments) g_pixel_segments[pix] += (uint32_t)(st.segments - seg0);
            if (J.normal && J.spp > 0) {
                J.normal[pix * 3 + 0] = last.normal.x;
                J.normal[pix * 3 + 1] = last.normal.y;
                J.normal[pix * 3 + 2] = last.normal.z;
            }
            if (J.depthbuf && J.spp > 0) J.depthbuf[pix] = last.depth;
            for (int k = 0; k < 5; ++k) J.rng[k * npix + pix] = s.v[k];
            J.rng[5 * npix + pix] = s.d;
        }
    }
}

}  // namespace

// =======================================================================================
// extern "C" surface for tests / bench cpu_baseline (ctypes).
// =======================================================================================
extern "C" {

int or_abi_version(void) { return 1; }

// DIAGNOSTIC: per-pixel segment counts of the following renders are ADDED to `out`
// ([n_rows * W] of the render's frame); nullptr turns it off.
void or_set_pixel_segments(uint32_t* out) { g_pixel_segments = out; }

// DIAGNOSTIC: per-pass draws and segments of the following renders ([n_rows * W][spp] each);
// nullptr turns it off.
void or_set_pass_trace(uint8_t* draws, uint8_t* segs) { g_pass_draws = draws; g_pass_segs = segs; }

// Binds texels to a material texture handle (replaces an earlier binding of the handle).
void or_bind_texture(uint64_t handle, const uint8_t* rgba, int w, int h, int valid_cols, int addr, int filter) {
    TexRec* t = new TexRec;
    t->rgba.assign(rgba, rgba + (size_t)valid_cols * h * 4);
    t->env = Env{nullptr, w, h, valid_cols, addr, filter};
    t->env.rgba = t->rgba.empty() ? nullptr : t->rgba.data();
    std::lock_guard<std::mutex> g(g_tex_mu);
    for (auto& e : g_textures)
        if (e.first == handle) { delete e.second; e.second = t; return; }
    g_textures.emplace_back(handle, t);
}

void or_clear_textures(void) {
    std::lock_guard<std::mutex> g(g_tex_mu);
    for (auto& e : g_textures) delete e.second;
    g_textures.clear();
}

uint64_t or_last_fallbacks(void) { return g_last_fallbacks; }

void or_set_walk(int ordered) { g_walk_ordered = ordered ? 1 : 0; }   // diagnostic, see trace_ray_ordered

int or_sizeof(int which) {
    switch (which) {
        case 0: return (int)sizeof(Material);
        case 1: return (int)sizeof(Object);
        case 2: return (int)sizeof(Camera);
        default: return -1;
    }
}

// --- detmath KAT surface -------------------------------------------------------------
double or_pow(double x, double y) { return dm_pow(x, y); }
double or_log(double x) { return dm_log(x); }
double or_exp(double x) { return dm_exp(x); }
double or_atan(double x) { return dm_atan(x); }
float or_powf(float x, float y) { return dm_powf(x, y); }
float or_sinf(float x) { return dm_sinf(x); }
float or_cosf(float x) { return dm_cosf(x); }
float or_asinf(float x) { return dm_asinf(x); }
float or_atanf(float x) { return dm_atanf(x); }

// Vectorised forms (op: 0 powf(a,b) 1 sinf 2 cosf 3 asinf 4 atanf 5 pow(a,b) as float of double).
void or_math_batch(int op, const float* a, const float* b, float* out, long n) {
    for (long i = 0; i < n; ++i) {
        switch (op) {
            case 0: out[i] = dm_powf(a[i], b[i]); break;
            case 1: out[i] = dm_sinf(a[i]); break;
            case 2: out[i] = dm_cosf(a[i]); break;
            case 3: out[i] = dm_asinf(a[i]); break;
            case 4: out[i] = dm_atanf(a[i]); break;
            case 5: out[i] = (float)dm_pow((double)a[i], 1.0 / (double)b[i]); break;
            case 9: out[i] = dm_pow5f(a[i]); break;
            default: out[i] = NAN;
        }
    }
}

// --- RNG -------------------------------------------------------------------------------
void or_curand_init(uint64_t seed, uint64_t subsequence, uint32_t out6[6]) {
    Xorwow s = curand_init(seed, subsequence);
    std::memcpy(out6, s.v, 20);
    out6[5] = s.d;
}

uint32_t or_xorwow_next(uint32_t st6[6]) {
    Xorwow s;
    std::memcpy(s.v, st6, 20);
    s.d = st6[5];
    uint32_t r = xorwow_next(s);
    std::memcpy(st6, s.v, 20);
    st6[5] = s.d;
    return r;
}

float or_uniform(uint32_t st6[6]) {
    Xorwow s;
    std::memcpy(s.v, st6, 20);
    s.d = st6[5];
    float r = uniform(s);
    std::memcpy(st6, s.v, 20);
    st6[5] = s.d;
    return r;
}

// A^(2^67 * 4^t) in rocRAND layout (compare: h_xorwow_sequence_jump_matrices[t]).
void or_seq_jump_matrix_pow4(int t, uint32_t out[800]) {
    const JumpTables& J = jump_tables();
    std::memcpy(out, J.seq[2 * t].m, sizeof(uint32_t) * 800);
}

// A^(4^t) in rocRAND layout (compare: h_xorwow_jump_matrices[t]) — pins the transition.
void or_jump_matrix_pow4(int t, uint32_t out[800]) {
    BitMat A;
    for (int c = 0; c < 160; ++c) {
        Xorwow s{};
        s.v[c / 32] = 1u << (c % 32);
        xorwow_next(s);
        std::memcpy(&A.m[c * 5], s.v, 20);
    }
    for (int i = 0; i < 2 * t; ++i) A = matmul(A, A);
    std::memcpy(out, A.m, sizeof(uint32_t) * 800);
}

// InitCuRand (path_tracer.cu:36-42): per pixel curand_init(seed, (x<<32)|y, 0).
void or_init_rng(uint64_t seed, int width, const int32_t* rows, int n_rows, uint32_t* rng_planar, int nthreads) {
    jump_tables();
    const size_t npix = (size_t)n_rows * width;
    if (nthreads < 1) nthreads = 1;
    auto work = [&](int t) {
        for (int ri = t; ri < n_rows; ri += nthreads)
            for (int x = 0; x < width; ++x) {
                Xorwow s = curand_init(seed, ((uint64_t)x << 32) | (uint64_t)(uint32_t)rows[ri]);
                size_t pix = (size_t)ri * width + x;
                for (int k = 0; k < 5; ++k) rng_planar[k * npix + pix] = s.v[k];
                rng_planar[5 * npix + pix] = s.d;
            }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
}

// --- Camera ---------------------------------------------------------------------------
// MotionalCamera::GetCopy (motional_camera.cu:177-200): basis + corner vectors; increments
// cur_sample_idx.  theta uses the double M_PI; tan of a float resolves to tanf.
void or_camera_get_copy(void* cam_inout) {
    Camera& c = *reinterpret_cast<Camera*>(cam_inout);
    float theta = (float)((double)c.view_fov * REF_PI / 180);
    float aspect = float(c.width) / float(c.height);
    float half_height = tanf(theta / 2);
    float half_width = aspect * half_height;
    c.w = normalize(sub(c.origin, c.look_at));
    c.u = normalize(cross(c.vup, c.w));
    c.v = cross(c.w, c.u);
    c.dist_to_focus = length(sub(c.origin, c.look_at));
    // top_left = origin - hw*d*u + hh*d*v - d*w, evaluated left to right:
    c.top_left = sub(add(sub(c.origin, mul(half_width * c.dist_to_focus, c.u)), mul(half_height * c.dist_to_focus, c.v)),
                     mul(c.dist_to_focus, c.w));
    c.horizontal = mul(2 * half_width * c.dist_to_focus, c.u);
    c.vertical = mul(-2 * half_height * c.dist_to_focus, c.v);
    c.cur_sample_idx++;
}

// --- BVH (topology export for tests) ----------------------------------------------------
// out: per node {bmin xyz, bmax xyz} floats (6) and {is_object, left, right, obj} ints (4).
int or_build_bvh(const void* objs, int n, float* out_box, int32_t* out_link, int cap) {
    Bvh b;
    build_bvh(b, reinterpret_cast<const Object*>(objs), n);
    int m = (int)b.nodes.size();
    for (int i = 0; i < m && i < cap; ++i) {
        const Node& nd = b.nodes[i];
        float* bx = out_box + i * 6;
        bx[0] = nd.bmin.x; bx[1] = nd.bmin.y; bx[2] = nd.bmin.z;
        bx[3] = nd.bmax.x; bx[4] = nd.bmax.y; bx[5] = nd.bmax.z;
        int32_t* l = out_link + i * 4;
        l[0] = nd.is_object; l[1] = nd.left; l[2] = nd.right; l[3] = nd.obj;
    }
    return m;
}

// --- Integrator -------------------------------------------------------------------------
// Renders `spp` passes of SamplePixel for every pixel of the given rows.  rng_planar is
// [6][n_rows*W] (in/out), accum is [n_rows*W][4] rgb-sum + pass count (in/out when
// accumulate != 0).  stats5 (optional) receives segments, node visits, primitive tests,
// hits, misses.  Returns 0 on success.
static int render_with(Bvh& bvh, const void* camera, const uint8_t* env_rgba, int env_w, int env_h,
                       int env_valid_cols, const int32_t* rows, int n_rows, int spp, int max_depth,
                       uint32_t* rng_planar, float* accum, float* normal_out, float* depth_out, uint64_t* stats5,
                       int accumulate, int nthreads) {
    RenderJob J;
    J.bvh = &bvh;
    J.env = Env{env_rgba, env_w, env_h, env_valid_cols};
    std::memcpy(&J.cam, camera, sizeof(Camera));
    J.rows = rows; J.n_rows = n_rows; J.spp = spp; J.max_depth = (uint32_t)max_depth;
    J.rng = rng_planar; J.accum = accum; J.normal = normal_out; J.depthbuf = depth_out;
    J.accumulate = accumulate;
    if (nthreads < 1) nthreads = 1;
    std::vector<Stats> st(nthreads, Stats{0, 0, 0, 0, 0, 0});
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t) th.emplace_back([&, t] { render_rows(J, t, nthreads, st[t]); });
    render_rows(J, 0, nthreads, st[0]);
    for (auto& x : th) x.join();
    if (stats5) {
        Stats s{0, 0, 0, 0, 0, 0};
        for (auto& x : st) { s.segments += x.segments; s.nodes += x.nodes; s.prims += x.prims; s.hits += x.hits; s.misses += x.misses; }
        stats5[0] = s.segments; stats5[1] = s.nodes; stats5[2] = s.prims; stats5[3] = s.hits; stats5[4] = s.misses;
    }
    uint64_t fb = 0;
    for (auto& x : st) fb += x.fallbacks;
    g_last_fallbacks = fb;
    return 0;
}

int or_render(const void* objs, int n_objs, const void* camera, const uint8_t* env_rgba, int env_w, int env_h,
              int env_valid_cols, const int32_t* rows, int n_rows, int spp, int max_depth, uint32_t* rng_planar,
              float* accum, float* normal_out, float* depth_out, uint64_t* stats5, int accumulate, int nthreads) {
    if (max_depth < 0 || max_depth > (int)MAX_RECURSION_DEPTH_SET) return -1;
    Bvh bvh;
    build_bvh(bvh, reinterpret_cast<const Object*>(objs), n_objs);
    return render_with(bvh, camera, env_rgba, env_w, env_h, env_valid_cols, rows, n_rows, spp, max_depth, rng_planar,
                       accum, normal_out, depth_out, stats5, accumulate, nthreads);
}

// Same as or_render, on a BVH built from `objs` and then edited by SceneBVH::UpdateObject
// (bvh.cu:122-157): edit k replaces object edit_idx[k] by edit_objs[k], then refits the
// leaf's box and every ancestor's box (MIN/MAX of its two children) up to the root.  The
// topology (and so the traversal order) stays the one of the original build.
// The diagnostic ordered walk's tree: walk_rebuild = 0 refits it the same way (the walk leaf
// takes the object's new box, its ancestors the MIN/MAX of their two children, left first:
// libcpt's device refit, cpt_kernels.hip k_refit_nodes); 1 rebuilds it from the edited objects
// (cpt_update_objects_rebuild).  A platform edit that changes whether the object is a platform
// always rebuilds (the walk tree holds only the bounded primitives).
int or_render_edited_ex(const void* objs, int n_objs, const int32_t* edit_idx, const void* edit_objs, int n_edits,
                        const void* camera, const uint8_t* env_rgba, int env_w, int env_h, int env_valid_cols,
                        const int32_t* rows, int n_rows, int spp, int max_depth, uint32_t* rng_planar, float* accum,
                        uint64_t* stats5, int nthreads, int walk_rebuild) {
    if (max_depth < 0 || max_depth > (int)MAX_RECURSION_DEPTH_SET) return -1;
    std::vector<Object> cur(reinterpret_cast<const Object*>(objs), reinterpret_cast<const Object*>(objs) + n_objs);
    Bvh bvh;
    build_bvh(bvh, cur.data(), n_objs);
    std::vector<int> parent(bvh.nodes.size(), -1), leaf_of(n_objs, -1);
    for (size_t i = 0; i < bvh.nodes.size(); ++i) {
        const Node& n = bvh.nodes[i];
        if (n.is_object) leaf_of[n.obj] = (int)i;
        else { parent[n.left] = (int)i; parent[n.right] = (int)i; }
    }
    std::vector<int> wparent(bvh.walk.size(), -1), wleaf_of(n_objs, -1);
    for (size_t i = 0; i < bvh.walk.size(); ++i) {
        const Bvh::WNode& n = bvh.walk[i];
        if (n.obj >= 0) wleaf_of[n.obj] = (int)i;
        else { wparent[n.left] = (int)i; wparent[n.right] = (int)i; }
    }
    const Object* E = reinterpret_cast<const Object*>(edit_objs);
    for (int k = 0; k < n_edits; ++k) {
        int o = edit_idx[k];
        if (o < 0 || o >= n_objs) return -2;
        if ((cur[o].type == PRIM_PLATFORM) != (E[k].type == PRIM_PLATFORM)) walk_rebuild = 1;
        cur[o] = E[k];
        for (int wi = wleaf_of[o]; wi != -1; wi = wparent[wi]) {   // the walk tree, refit alike
            Bvh::WNode& n = bvh.walk[wi];
            if (n.obj >= 0) {
                n.bmax = aabb_max(cur[n.obj]);
                n.bmin = aabb_min(cur[n.obj]);
            } else {
                const Bvh::WNode& L = bvh.walk[n.left];
                const Bvh::WNode& R = bvh.walk[n.right];
                n.bmax = mk(MAX_(L.bmax.x, R.bmax.x), MAX_(L.bmax.y, R.bmax.y), MAX_(L.bmax.z, R.bmax.z));
                n.bmin = mk(MIN_(L.bmin.x, R.bmin.x), MIN_(L.bmin.y, R.bmin.y), MIN_(L.bmin.z, R.bmin.z));
            }
        }
        for (int ni = leaf_of[o]; ni != -1; ni = parent[ni]) {      // UpdateSceneBVH (bvh.cu:122-141)
            Node& n = bvh.nodes[ni];
            if (n.is_object) {
                n.bmax = aabb_max(cur[n.obj]);
                n.bmin = aabb_min(cur[n.obj]);
            } else {
                const Node& L = bvh.nodes[n.left];
                const Node& R = bvh.nodes[n.right];
                n.bmax = mk(MAX_(L.bmax.x, R.bmax.x), MAX_(L.bmax.y, R.bmax.y), MAX_(L.bmax.z, R.bmax.z));
                n.bmin = mk(MIN_(L.bmin.x, R.bmin.x), MIN_(L.bmin.y, R.bmin.y), MIN_(L.bmin.z, R.bmin.z));
            }
        }
    }
    if (walk_rebuild) build_walk_tree(bvh);
    return render_with(bvh, camera, env_rgba, env_w, env_h, env_valid_cols, rows, n_rows, spp, max_depth, rng_planar,
                       accum, nullptr, nullptr, stats5, 0, nthreads);
}

int or_render_edited(const void* objs, int n_objs, const int32_t* edit_idx, const void* edit_objs, int n_edits,
                     const void* camera, const uint8_t* env_rgba, int env_w, int env_h, int env_valid_cols,
                     const int32_t* rows, int n_rows, int spp, int max_depth, uint32_t* rng_planar, float* accum,
                     uint64_t* stats5, int nthreads) {
    return or_render_edited_ex(objs, n_objs, edit_idx, edit_objs, n_edits, camera, env_rgba, env_w, env_h,
                               env_valid_cols, rows, n_rows, spp, max_depth, rng_planar, accum, stats5, nthreads, 0);
}

// Denoising + Mix (path_tracer.cu:177-254) for a full W x H frame.  radiance = accum rgb /
// pass count; neighbours by linear offset over the W' x H' = 16*floor(W/16) x 16*floor(H/16)
// launch (rows wrap); weights in double; mix = lerp(mix, clamp(dn, 0, 1), 1/idx); bytes
// 0..2 = 255.99*(b, g, r); alpha untouched.
// The same for output rows [y0, y1) only: accum/normal/depth hold rows row0.. (stride W; they
// must include every row the stencil reaches, y0 - 3 .. y1 + 2 within [0, H')), mix/out hold
// the band's rows.  Row-banded multi-GPU display.
void or_denoise_mix_band(const float* accum, const float* normal, const float* depth, float* mix, uint8_t* out,
                         int W, int H, int row0, int y0, int y1, uint32_t cur_sample_idx);

void or_denoise_mix(const float* accum, const float* normal, const float* depth, float* mix, uint8_t* out, int W,
                    int H, uint32_t cur_sample_idx) {
    or_denoise_mix_band(accum, normal, depth, mix, out, W, H, 0, 0, 16 * (H / 16), cur_sample_idx);
}

void or_denoise_mix_band(const float* accum, const float* normal, const float* depth, float* mix, uint8_t* out,
                         int W, int H, int row0, int y0, int y1, uint32_t cur_sample_idx) {
    const int we = 16 * (W / 16), he = 16 * (H / 16);
    const float kernel[5][5] = {{1.f, 4.f, 7.f, 4.f, 1.f},
                                {4.f, 16.f, 26.f, 16.f, 4.f},
                                {7.f, 26.f, 41.f, 26.f, 7.f},
                                {4.f, 16.f, 26.f, 16.f, 4.f},
                                {1.f, 4.f, 7.f, 4.f, 1.f}};
    auto rad = [&](int px) {
        const float* a = accum + 4 * (size_t)px;
        return a[3] != 0.f ? divs(mk(a[0], a[1], a[2]), a[3]) : mk(a[0], a[1], a[2]);
    };
    auto nrm = [&](int px) { return mk(normal[3 * px], normal[3 * px + 1], normal[3 * px + 2]); };
    auto wgt = [](float d2) {
        double w = dm_exp(-((double)d2) / REF_PI);   // min(exp(-d2/M_PI), 1.0)
        return (float)(w < 1.0 ? w : 1.0);
    };
    const float inv_idx = 1.f / float(cur_sample_idx);
    if (we == 0) return;
    for (int y = y0; y < y1 && y < he; ++y)
        for (int x = 0; x < we; ++x) {
            const int self = (y - row0) * W + x, bself = (y - y0) * W + x;
            f3 cval = rad(self), nval = nrm(self);
            float pval = depth[self];
            f3 sum = mk1(0.f);
            float cum_w = 0.0f;
            for (int i = 0; i < 5; ++i)
                for (int j = 0; j < 5; ++j) {
                    int u = x + (i - 2), v = y + (j - 2);
                    int cur_off = v * we + u;
                    float weight;
                    f3 ctmp;
                    if (cur_off < 0 || cur_off >= we * he) {
                        weight = 0.f;
                        ctmp = mk1(0.f);
                    } else {
                        int px = (cur_off / we - row0) * W + (cur_off % we);
                        ctmp = rad(px);
                        f3 t = sub(cval, ctmp);
                        float c_w = wgt(dot(t, t));
                        t = sub(nval, nrm(px));
                        double dn = (double)dot(t, t);
                        float n_w = wgt((float)(dn > 0.0 ? dn : 0.0));
                        float ptmp = depth[px];
                        float p_w = wgt((pval - ptmp) * (pval - ptmp));
                        weight = c_w * n_w * p_w;
                    }
                    sum = add(sum, mul(weight * kernel[i][j], ctmp));
                    cum_w += weight * kernel[i][j];
                }
            f3 dn = divs(sum, cum_w);
            f3 cl = mk(fmaxf(0.f, fminf(dn.x, 1.f)), fmaxf(0.f, fminf(dn.y, 1.f)), fmaxf(0.f, fminf(dn.z, 1.f)));
            float* m = mix + 3 * (size_t)bself;
            f3 mv = mk(m[0], m[1], m[2]);
            mv = add(mv, mul(inv_idx, sub(cl, mv)));
            m[0] = mv.x; m[1] = mv.y; m[2] = mv.z;
            out[4 * (size_t)bself + 0] = (uint8_t)(255.99f * mv.z);
            out[4 * (size_t)bself + 1] = (uint8_t)(255.99f * mv.y);
            out[4 * (size_t)bself + 2] = (uint8_t)(255.99f * mv.x);
        }
}

}  // extern "C"
