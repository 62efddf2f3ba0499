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
