"""Exact replacements the device code uses instead of slower IEEE sequences (cpt_device.hpp
dm::div_pi -- also under the display's pair weights, cpt_kernels.hip dn_weight --, dm::div255; cpt_path.hpp mirror_index's division-free range).  Each must return
the bit pattern of the expression it replaces, checked here exhaustively on the host: the
formulas are plain IEEE double operations (fma included), which the GPU executes alike."""
import os
import subprocess

import numpy as np
import pytest

SRC = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static const double REF_PI = 3.14159265358979323846;
static double div_pi(float a) {
    const double INV_PI = 1.0 / REF_PI;
    const double q = (double)a * INV_PI;
    if (q == 0.0) return q;
    const double r = fma(-q, REF_PI, (double)a);
    return fma(r, INV_PI, q);
}
static int mirror_general(int i, int n) {
    int period = 2 * n, m = i % period;
    if (m < 0) m += period;
    if (m >= n) m = period - 1 - m;
    return m;
}
static int mirror_fast(int i, int n) {
    int m = i < 0 ? -1 - i : i;
    return m >= n ? 2 * n - 1 - m : m;
}
int main(void) {
    unsigned long long bad = 0, n = 0;
    /* every float in [-2, 2]: bit patterns 0 .. 0x40000000 and their negatives */
    for (uint32_t b = 0; b <= 0x40000000u; ++b) {
        for (int s = 0; s < 2; ++s) {
            uint32_t bb = b | (s ? 0x80000000u : 0u);
            float a; memcpy(&a, &bb, 4);
            double x = div_pi(a), y = (double)a / REF_PI;
            if (memcmp(&x, &y, 8) != 0) { if (bad < 5) printf("div_pi %a\n", a); bad++; }
            n++;
        }
    }
    /* the denoise weights' range (cpt_kernels.hip dn_weight): every float in [2, 2341); from
       2341 on, exp(-x / pi) is below exp's underflow bound and dn_weight returns 0 directly */
    {
        float lim = 2341.0f;
        uint32_t lb; memcpy(&lb, &lim, 4);
        for (uint32_t b = 0x40000000u; b < lb; ++b) {
            float a; memcpy(&a, &b, 4);
            double x = div_pi(a), y = (double)a / REF_PI;
            if (memcmp(&x, &y, 8) != 0) { if (bad < 5) printf("div_pi %a\n", a); bad++; }
            n++;
        }
        if (!((double)lim / REF_PI > 745.1332191019412)) { printf("dn_weight bound\n"); bad++; }
    }
    for (uint32_t k = 0; k < 256; ++k) {
        float x = (float)((double)k * (1.0 / 255.0)), y = (float)k / 255.0f;
        if (memcmp(&x, &y, 4) != 0) { printf("div255 %u\n", k); bad++; }
    }
    int sizes[] = {1, 2, 3, 7, 320, 1280, 2048, 4096};
    for (int t = 0; t < 8; ++t) {
        int w = sizes[t];
        for (int i = -w; i < 2 * w; ++i)
            if (mirror_fast(i, w) != mirror_general(i, w)) { printf("mirror %d %d\n", i, w); bad++; }
    }
    printf("checked %llu bad %llu\n", n, bad);
    return bad != 0;
}
"""


def test_exact_identities(tmp_path):
    src = tmp_path / "ident.c"
    exe = tmp_path / "ident"
    src.write_text(SRC)
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-o", str(exe), str(src), "-lm"],
                   check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout
    assert "bad 0" in r.stdout
    print(r.stdout)


# The display's pair weight against the oracle's own expression min(exp(-(double)d2 / M_PI), 1.0)
# stored to float (oracle or_exp = dm_exp, path_tracer.cu:224,228,231), for every float d2 in
# [0, 2341] and the special values: the round-4 branch-free form (cpt_kernels.hip dn_weight_slow:
# the quotient, dm_exp's steps with a plain ldexp below x = -105.05, the shortcuts 0 -> 1,
# >= 330 -> 0), and the round-5 short form (dn_weight: the 2^(-j/32) table exp of
# cpt_dn_exp.hpp and the rounding guard that falls back to the slow form).  The harness calls the
# oracle library (test infrastructure).
DN_SRC = r"""
#include "cpt_dn_exp.hpp"
#include <dlfcn.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static const double REF_PI = 3.14159265358979323846;
static const double LN2_HI = 6.93147180369123816490e-01, LN2_LO = 1.90821492927058770002e-10;
static const double INV_LN2 = 1.44269504088896338700e+00;
static double (*or_exp)(double);
static float ref_w(float d2) {
    double w = or_exp(-((double)d2) / REF_PI);
    return (float)(w < 1.0 ? w : 1.0);
}
static float fast_w(float d2) {   /* cpt_kernels.hip dn_weight, operation for operation */
    const double INV_PI = 1.0 / REF_PI;
    const double a = (double)d2, q = a * INV_PI;
    const double x = -fma(fma(-q, REF_PI, a), INV_PI, q);
    const double k = floor(fma(x, INV_LN2, 0.5));
    const double r = fma(-k, LN2_LO, fma(-k, LN2_HI, x));
    double p = 1.0 / 6227020800.0;
    const double c[13] = {1.0 / 479001600.0, 1.0 / 39916800.0, 1.0 / 3628800.0, 1.0 / 362880.0, 1.0 / 40320.0,
                          1.0 / 5040.0, 1.0 / 720.0, 1.0 / 120.0, 1.0 / 24.0, 1.0 / 6.0, 0.5, 1.0, 1.0};
    for (int i = 0; i < 13; ++i) p = fma(r, p, c[i]);
    int ki = (k == k) ? (int)k : 0;    /* (the device's cvt of a NaN: any k, ldexp(NaN) stays NaN) */
    const double w = ldexp(p, ki);
    float f = (float)(w < 1.0 ? w : 1.0);
    f = d2 >= 330.0f ? 0.0f : f;
    return d2 == 0.0f ? 1.0f : f;
}
static const double DN_TAB[cpt::DN_EXP_N] = CPT_DN_EXP_TABLE_INIT;
static int g_guard_fallbacks[8];
static float short_w(float d2, int t) {   /* cpt_kernels.hip dn_exp_short + dn_weight */
    const double SHIFT = 0x1.8p52, a = (double)d2;
    const double tt = fma(a, cpt::DN_KN_HI, SHIFT), nd = tt - SHIFT;
    uint64_t tb; memcpy(&tb, &tt, 8);
    const uint32_t n = (uint32_t)tb;
    double r = fma(a, cpt::DN_KN_HI, -nd);
    r = fma(a, cpt::DN_KN_LO, r);
    double p = cpt::DN_POLY_DEG >= 4 ? (cpt::DN_POLY_DEG >= 5 ? fma(r, cpt::DN_C5, cpt::DN_C4) : cpt::DN_C4) : cpt::DN_C3;
    if (cpt::DN_POLY_DEG >= 4) p = fma(r, p, cpt::DN_C3);
    p = fma(r, p, cpt::DN_C2);
    p = fma(r, p, cpt::DN_C1);
    p = fma(r, p, 1.0);
    double T = DN_TAB[n & (uint32_t)(cpt::DN_EXP_N - 1)];
    uint64_t Tb; memcpy(&Tb, &T, 8);
    const uint32_t hi = (uint32_t)(Tb >> 32) - ((n >> cpt::DN_EXP_SHIFT) << 20);
    Tb = ((uint64_t)hi << 32) | (Tb & 0xffffffffull);
    memcpy(&T, &Tb, 8);
    const double e = T * p;
    uint64_t eb; memcpy(&eb, &e, 8);
    const uint32_t elo = (uint32_t)eb, ehi = (uint32_t)(eb >> 32);
    const int dm = (int)(elo & 0x1fffffffu) - (1 << 28);
    const bool normal_f = ehi >= 0x38100000u && ehi <= 0x3ff00000u;
    const bool near = !normal_f || (dm < 512 && dm > -512);
    float f = (float)e;
    if (near && !(d2 >= 330.0f)) { f = fast_w(d2); if (t >= 0) g_guard_fallbacks[t]++; }
    f = d2 >= 330.0f ? 0.0f : f;
    return d2 == 0.0f ? 1.0f : f;
}
static uint32_t g_lim;
static unsigned long long g_bad[8];
static void* run(void* arg) {
    int t = (int)(intptr_t)arg;
    for (uint32_t b = (uint32_t)t; b <= g_lim; b += 8) {
        float d; memcpy(&d, &b, 4);
        float x = ref_w(d), y = fast_w(d), z = short_w(d, t);
        if (memcmp(&x, &y, 4) != 0) { if (g_bad[t] < 3) printf("dn_weight_slow %a: %a vs %a\n", d, x, y); g_bad[t]++; }
        if (memcmp(&x, &z, 4) != 0) { if (g_bad[t] < 3) printf("dn_weight %a: %a vs %a\n", d, x, z); g_bad[t]++; }
    }
    return 0;
}
int main(int argc, char** argv) {
    void* h = dlopen(argv[1], RTLD_NOW);
    if (!h) { printf("dlopen failed\n"); return 2; }
    or_exp = (double (*)(double))dlsym(h, "or_exp");
    float lim = 2341.0f; memcpy(&g_lim, &lim, 4);
    pthread_t th[8];
    for (int t = 0; t < 8; ++t) pthread_create(&th[t], 0, run, (void*)(intptr_t)t);
    unsigned long long bad = 0;
    for (int t = 0; t < 8; ++t) { pthread_join(th[t], 0); bad += g_bad[t]; }
    const float sp[] = {INFINITY, NAN, -0.0f, 3.4e38f, 1e-45f, 329.99998f, 330.0f, 2340.9f};
    for (int i = 0; i < 8; ++i) {
        float x = ref_w(sp[i]), y = fast_w(sp[i]), z = short_w(sp[i], -1);
        if (memcmp(&x, &y, 4) != 0) { printf("special %a: %a vs %a\n", sp[i], x, y); bad++; }
        if (memcmp(&x, &z, 4) != 0) { printf("special short %a: %a vs %a\n", sp[i], x, z); bad++; }
    }
    long fb = 0;
    for (int t = 0; t < 8; ++t) fb += g_guard_fallbacks[t];
    printf("guard fallbacks %ld of %u\n", fb, g_lim + 1);
    printf("bad %llu\n", bad);
    return bad != 0;
}
"""


def test_denoise_weight_exhaustive(tmp_path):
    import oracle
    lib = oracle.build()
    src = tmp_path / "dnw.cpp"
    exe = tmp_path / "dnw"
    src.write_text(DN_SRC)
    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cpppathtracer_amd", "csrc")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-fno-fast-math", "-I", csrc, "-o", str(exe), str(src), "-lm",
                    "-ldl", "-lpthread"], check=True)
    r = subprocess.run([str(exe), lib], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout
    assert "bad 0" in r.stdout
    print(r.stdout)
