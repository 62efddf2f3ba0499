// cpt_host_rng.cpp — InitCuRand's host half (path_tracer.cu:36-42): the XORWOW transition's
// GF(2) jump tables and curand_init's seed scrambling (cpt_host.hpp).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <functional>
#include <mutex>
#include <queue>
#include <vector>

#include "cpt_host.hpp"

namespace cpt {
namespace host {

// ------------------------------------------------------------------------------------
// XORWOW jump tables: jumps[t] = A^(2^67 * 2^t), 160x160 over GF(2), column-major
// (column c = A^k e_c as 5 words), the layout rocRAND uses (rocrand_xorwow.h:51-65).
// ------------------------------------------------------------------------------------
namespace {
struct BitMat { uint32_t m[800]; };

void xorshift_step(uint32_t v[5]) {   // linear part of curand() (d excluded)
    uint32_t t = v[0] ^ (v[0] >> 2);
    v[0] = v[1]; v[1] = v[2]; v[2] = v[3]; v[3] = v[4];
    v[4] = (v[4] ^ (v[4] << 4)) ^ (t ^ (t << 1));
}

void bm_apply(const BitMat& M, const uint32_t in[5], uint32_t out[5]) {
    uint32_t r[5] = {0, 0, 0, 0, 0};
    for (int c = 0; c < 160; ++c)
        if ((in[c >> 5] >> (c & 31)) & 1u)
            for (int k = 0; k < 5; ++k) r[k] ^= M.m[c * 5 + k];
    std::memcpy(out, r, sizeof(r));
}

BitMat bm_square(const BitMat& M) {
    BitMat R;
    for (int c = 0; c < 160; ++c) bm_apply(M, &M.m[c * 5], &R.m[c * 5]);
    return R;
}

}  // namespace

const std::vector<uint32_t>& jump_tables() {
    static std::vector<uint32_t> tbl;
    static std::once_flag once;
    std::call_once(once, [] {
        BitMat A;
        for (int c = 0; c < 160; ++c) {
            uint32_t v[5] = {0, 0, 0, 0, 0};
            v[c >> 5] = 1u << (c & 31);
            xorshift_step(v);
            std::memcpy(&A.m[c * 5], v, 20);
        }
        for (int i = 0; i < 67; ++i) A = bm_square(A);
        tbl.resize(64 * 800);
        for (int t = 0; t < 64; ++t) {
            std::memcpy(&tbl[(size_t)t * 800], A.m, sizeof(A.m));
            A = bm_square(A);
        }
    });
    return tbl;
}

// curand_init's seed scrambling (curand_kernel.h, CUDA 11.7).
void curand_seed_state(uint64_t seed, uint32_t out[6]) {
    uint32_t s0 = (uint32_t)seed ^ 0xaad26b49u;
    uint32_t s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
    uint32_t t0 = 1099087573u * s0;
    uint32_t t1 = 2591861531u * s1;
    out[0] = 123456789u + t0;
    out[1] = 362436069u ^ t0;
    out[2] = 521288629u + t1;
    out[3] = 88675123u ^ t1;
    out[4] = 5783321u + t0;
    out[5] = 6615241u + t1 + t0;
}

}  // namespace host
}  // namespace cpt
