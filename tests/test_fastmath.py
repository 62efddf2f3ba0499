"""The BSDF lobe's short transcendentals (cpt_device.hpp fm::pow_unit, fm::sincos_2pi, lobe_pow,
lobe_sincos; round 6) restated on the host operation for operation and checked against the
oracle's full sequences (or_pow, or_sinf, or_cosf: dm_pow / dm_sinf / dm_cosf, the restatement of
material.cu:24-27,43-48,78-86,104-105's pow / cosf / sinf), float for float:

* Diffuse's (float)pow(x, 0.5) == sqrtf(x) for every float x in [2^-42, 1] (the lobe's x_1 =
  curand_uniform >= 2^-33); below 2^-42 the identity fails for 23 floats, so lobe_pow keeps
  the full pow there;
* lobe_pow(x, y) == (float)pow(x, y) for every float x in [2^-33, 1] at one of S4's exponents,
  every 7th normal float at S4's others, and every 61st float of (0, 1] at the S1000 materials'
  and edge exponents of the short form's domain;
* lobe_sincos(phi) == (sinf(phi), cosf(phi)) for every float phi in [0, 2 pi];
* the sky fetch's miss_atanf / miss_asinf (fm::atan_ratio, path_tracer.cu:119-120) == atanf /
  asinf on every 31st float / every 7th float in [-1, 1] (the host form uses IEEE quotients where the
  device takes hardware reciprocal estimates; the device test checks the shipped code).

Also reports how often the rounding guard sends an input to the full sequence.  The device
code itself is checked against the device's full sequences for every float of the same domains
(test_gpu_parity.py::test_lobe_*_exhaustive).  The harness calls the oracle library (test
infrastructure)."""
import os
import subprocess

import numpy as np
import pytest
from conftest import lobe_exponents

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cpppathtracer_amd", "csrc")

SRC = r"""
#include "cpt_fm_tables.hpp"
#include <dlfcn.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
using namespace cpt;
static double (*or_pow)(double, double);
static float (*or_sinf)(float);
static float (*or_cosf)(float);
static float (*or_atanf)(float);
static float (*or_asinf)(float);
static const double LOG_TAB[2 * FM_LOG_N] = CPT_FM_LOG_TABLE_INIT;
static const double EXP_TAB[FM_EXP_N] = CPT_FM_EXP_TABLE_INIT;
static const double SC_TAB[2 * (2 * FM_SC_N + 1)] = CPT_FM_SC_TABLE_INIT;
static uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float bitsf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint64_t dbits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
static double bitsd(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
static bool sure_f32(double d) {   /* cpt_device.hpp fm::sure_f32 */
    const uint64_t b = dbits(d);
    const uint32_t lo = (uint32_t)b, hi = (uint32_t)(b >> 32) & 0x7fffffffu;
    const int dm_ = (int)(lo & 0x1fffffffu) - (1 << 28);
    return hi - 0x38100000u < 0x07f00000u && (dm_ >= 1024 || dm_ <= -1024);
}
static double pow_unit(float x, double y, bool& ok) {   /* fm::pow_unit */
    const uint32_t ux = fbits(x);
    const int e = (int)(ux >> 23) - 127;
    const uint32_t i = (ux >> 16) & (uint32_t)(FM_LOG_N - 1);
    const double m = (double)bitsf((ux & 0x007fffffu) | 0x3f800000u);
    const double c = LOG_TAB[2 * i], lnc = LOG_TAB[2 * i + 1];
    const double r = fma(m, c, -1.0);
    double q = fma(r, FM_L6, FM_L5);
    q = fma(r, q, FM_L4);
    q = fma(r, q, FM_L3);
    q = fma(r, q, FM_L2);
    const double lp = fma(r * r, q, r);
    const double t = y * fma((double)e, FM_LN2, lnc + lp);
    const double SHIFT = 0x1.8p52;
    const double tt = fma(t, FM_KN_HI, SHIFT);
    const double nd = tt - SHIFT;
    const int n = (int)(uint32_t)dbits(tt);
    double s = fma(t, FM_KN_HI, -nd);
    s = fma(t, FM_KN_LO, s);
    double p = fma(s, FM_E4, FM_E3);
    p = fma(s, p, FM_E2);
    p = fma(s, p, FM_E1);
    p = fma(s, p, 1.0);
    const uint64_t Tb = dbits(EXP_TAB[n & (FM_EXP_N - 1)]);
    const uint32_t hi = (uint32_t)(Tb >> 32) + ((uint32_t)(n >> 7) << 20);
    const double Ts = bitsd(((uint64_t)hi << 32) | (Tb & 0xffffffffull));
    const double d = Ts * p;
    ok = ux - 0x00800000u <= 0x3f000000u && y > 0.0 && y <= 1.0 && t >= -2.0 && sure_f32(d);
    return d;
}
static void sincos_2pi(float phi, double& s, double& c, bool& ok) {   /* fm::sincos_2pi */
    const double x = (double)phi, SHIFT = 0x1.8p52;
    const double tt = fma(x, FM_SC_K, SHIFT);
    const double kd = tt - SHIFT;
    const uint32_t k = (uint32_t)dbits(tt);
    double r = fma(-kd, FM_SC_P1, x);
    r = fma(-kd, FM_SC_P2, r);
    const double r2 = r * r;
    double ps = fma(r2, FM_S7, FM_S5);
    ps = fma(r2, ps, FM_S3);
    const double sr = fma(r * r2, ps, r);
    double pc = fma(r2, FM_C6, FM_C4);
    pc = fma(r2, pc, FM_C2);
    const double cr = fma(r2, pc, 1.0);
    const uint32_t kk = k <= (uint32_t)(2 * FM_SC_N) ? k : 0u;
    const double S = SC_TAB[2 * kk], C = SC_TAB[2 * kk + 1];
    s = fma(S, cr, C * sr);
    c = fma(C, cr, -(S * sr));
    ok = phi >= 0.0f && phi <= 6.28318548f && sure_f32(s) && sure_f32(c);
}
static const double AT_TAB[2 * (FM_AT_N + 1)] = CPT_FM_AT_TABLE_INIT;
/* fm::atan_ratio, with the device's two hardware reciprocal estimates (v_rcp_f32 for k, v_rcp_f64
   before the two Newton steps) replaced by IEEE quotients: k may differ where the float ratio
   sits at a rounding tie and the double result in its last bits, so this restates the form and
   its guard, and the device test compares the shipped code itself */
static double atan_ratio(double n, double m, bool& ok) {
    const bool big = n > m;
    const float rf = (float)(big ? m : n) * (1.0f / (float)(big ? n : m));
    const float kf = fminf(rintf(32.0f * rf), 32.0f);
    const double c = (double)kf * 0.03125;
    const double num = big ? fma(-c, n, m) : fma(-c, m, n);
    const double den = big ? fma(c, m, n) : fma(c, n, m);
    double r = 1.0 / den;
    double e = fma(-den, r, 1.0);
    r = fma(r, e, r);
    const double d = num * r;
    const double d2 = d * d;
    double p = fma(d2, FM_A7, FM_A5);
    p = fma(d2, p, FM_A3);
    const double at = fma(d * d2, p, d);
    const int k = (int)kf;
    const double T = AT_TAB[2 * (k >= 0 && k <= FM_AT_N ? k : 0) + (big ? 1 : 0)];
    const double res = big ? T - at : T + at;
    ok = n >= 0.0 && m > 0.0 && sure_f32(res);
    return res;
}
static float lobe_pow(float x, double y, bool& fell) {   /* lobe_pow */
    fell = false;
    if (y == 0.5 && x >= 0x1p-42f) return sqrtf(x);
    bool ok;
    const double d = pow_unit(x, y, ok);
    if (ok) return (float)d;
    fell = true;
    return (float)or_pow((double)x, y);
}
static int g_mode, g_step;
static double g_y;
static uint32_t g_lo, g_hi;
static unsigned long long g_bad[8], g_fell[8], g_n[8];
static void* run(void* arg) {
    const int t = (int)(intptr_t)arg;
    for (uint64_t b = g_lo + (uint64_t)t * g_step; b <= g_hi; b += 8ull * g_step) {
        const float x = bitsf((uint32_t)b);
        g_n[t]++;
        if (g_mode == 0) {
            const float a = sqrtf(x), r = (float)or_pow((double)x, 0.5);
            if (fbits(a) != fbits(r)) { if (g_bad[t] < 3) printf("sqrt %a: %a vs %a\n", x, a, r); g_bad[t]++; }
        } else if (g_mode == 1) {
            bool fell;
            const float a = lobe_pow(x, g_y, fell), r = (float)or_pow((double)x, g_y);
            g_fell[t] += fell;
            if (fbits(a) != fbits(r)) { if (g_bad[t] < 3) printf("pow %a %a: %a vs %a\n", x, g_y, a, r); g_bad[t]++; }
        } else if (g_mode == 3) {   /* miss_atanf */
            bool ok;
            const double a = atan_ratio(fabs((double)x), 1.0, ok);
            float f = (float)(x < 0.0f ? -a : a);
            const float r = or_atanf(x);
            if (!ok) { f = r; g_fell[t]++; }
            if (fbits(f) != fbits(r)) { if (g_bad[t] < 3) printf("atanf %a: %a vs %a\n", x, f, r); g_bad[t]++; }
        } else if (g_mode == 4) {   /* miss_asinf */
            const double xd = (double)x;
            bool ok;
            const double a = atan_ratio(fabs(xd), sqrt((1.0 - xd) * (1.0 + xd)), ok);
            float f = (float)(x < 0.0f ? -a : a);
            const float r = or_asinf(x);
            if (!ok) { f = r; g_fell[t]++; }
            if (fbits(f) != fbits(r)) { if (g_bad[t] < 3) printf("asinf %a: %a vs %a\n", x, f, r); g_bad[t]++; }
        } else if (g_mode == 2) {
            double s, c;
            bool ok;
            sincos_2pi(x, s, c, ok);
            const float rs = or_sinf(x), rc = or_cosf(x);
            float as = (float)s, ac = (float)c;
            if (!ok) { as = rs; ac = rc; g_fell[t]++; }
            if (fbits(as) != fbits(rs) || fbits(ac) != fbits(rc)) {
                if (g_bad[t] < 3) printf("sincos %a: %a %a vs %a %a\n", x, as, ac, rs, rc);
                g_bad[t]++;
            }
        }
    }
    return 0;
}
/* argv: lib mode lo hi step [y] */
int main(int argc, char** argv) {
    void* h = dlopen(argv[1], RTLD_NOW);
    if (!h) { printf("dlopen failed\n"); return 2; }
    or_pow = (double (*)(double, double))dlsym(h, "or_pow");
    or_sinf = (float (*)(float))dlsym(h, "or_sinf");
    or_cosf = (float (*)(float))dlsym(h, "or_cosf");
    or_atanf = (float (*)(float))dlsym(h, "or_atanf");
    or_asinf = (float (*)(float))dlsym(h, "or_asinf");
    g_mode = atoi(argv[2]);
    g_lo = (uint32_t)strtoul(argv[3], 0, 0);
    g_hi = (uint32_t)strtoul(argv[4], 0, 0);
    g_step = atoi(argv[5]);
    g_y = argc > 6 ? strtod(argv[6], 0) : 0.0;
    pthread_t th[8];
    for (int t = 0; t < 8; ++t) pthread_create(&th[t], 0, run, (void*)(intptr_t)t);
    unsigned long long bad = 0, fell = 0, n = 0;
    for (int t = 0; t < 8; ++t) { pthread_join(th[t], 0); bad += g_bad[t]; fell += g_fell[t]; n += g_n[t]; }
    printf("checked %llu fallbacks %llu bad %llu\n", n, fell, bad);
    return bad != 0;
}
"""

X_2M42 = int(np.float32(2.0 ** -42).view(np.uint32))
X_ONE = int(np.float32(1.0).view(np.uint32))
X_2M33 = int(np.float32(2.0 ** -33).view(np.uint32))
X_MIN_NORMAL = 0x00800000
X_2PI = int(np.float32(2 * np.pi).view(np.uint32))   # (float)(2 pi) rounds up: the lobe's largest phi


@pytest.fixture(scope="module")
def fm_exe(tmp_path_factory):
    d = tmp_path_factory.mktemp("fm")
    src, exe = d / "fm.cpp", d / "fm"
    src.write_text(SRC)
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-fno-fast-math", "-I", CSRC, "-o", str(exe), str(src),
                    "-lm", "-ldl", "-lpthread"], check=True)
    return str(exe)


def _run(fm_exe, oracle_mod, *args):
    lib = oracle_mod.build()
    r = subprocess.run([fm_exe, lib, *[str(a) for a in args]], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout
    assert "bad 0" in r.stdout, r.stdout
    print(args, r.stdout.strip())
    n, fell = (int(v) for v in r.stdout.split()[1:4:2])
    return n, fell


def test_diffuse_pow_half_is_sqrtf(fm_exe, oracle_mod):
    _run(fm_exe, oracle_mod, 0, X_2M42, X_ONE, 1)


@pytest.mark.parametrize("smooth_idx", [0, 1, 2])
def test_lobe_pow_s4(fm_exe, oracle_mod, smooth_idx):
    """Every float of the lobe's x_1 range [2^-33, 1] at S4's first exponent, every 7th float of
    (0, 1] at the others (every float of (0, 1]: on the device)."""
    y = lobe_exponents(oracle_mod, "s4")[smooth_idx]
    if smooth_idx == 0:
        n, fell = _run(fm_exe, oracle_mod, 1, X_2M33, X_ONE, 1, y.hex())
    else:
        n, fell = _run(fm_exe, oracle_mod, 1, X_MIN_NORMAL, X_ONE, 7, y.hex())
    assert fell < 1e-5 * n


def test_lobe_pow_s1000_and_edges(fm_exe, oracle_mod):
    """Every 61st float of (0, 1] (subnormals included: the full pow decides) at the S1000
    materials' exponents and the edges of the short form's domain."""
    ys = lobe_exponents(oracle_mod, "s1000") + [1.0, 0.999, 0.25, 0.0625, 1e-3, 2.0 ** -40, 1e-300, 1.5, 0.0]
    for y in ys:
        _run(fm_exe, oracle_mod, 1, 1, X_ONE, 61, y.hex())


def test_lobe_sincos_exhaustive(fm_exe, oracle_mod):
    n, fell = _run(fm_exe, oracle_mod, 2, 0, X_2PI, 1)
    # 0 and the 2^23 - 1 subnormal phi (sin phi a subnormal float) always take the full sequence
    assert fell - X_MIN_NORMAL < 1e-5 * n


@pytest.mark.parametrize("sign", [0, 0x80000000])
def test_miss_atanf(fm_exe, oracle_mod, sign):
    """Every 31st float of either sign (the device test takes all 2^32)."""
    n, fell = _run(fm_exe, oracle_mod, 3, sign, sign + 0x7f800000, 31)
    # 0 and the subnormals (atan x = x: a subnormal float) always take the full sequence
    assert fell - X_MIN_NORMAL // 31 < 1e-5 * n


def test_miss_asinf(fm_exe, oracle_mod):
    """Every 7th float in [-1, 1] (the device test takes all 2^32)."""
    for lo in (0, 0x80000000):
        n, fell = _run(fm_exe, oracle_mod, 4, lo, lo + X_ONE, 7)
        assert fell - X_MIN_NORMAL // 7 < 1e-5 * n
