// cpt_stamps.hpp — DIAGNOSTIC wave-time stamps of the megakernel (CPT_STAMPS builds only; a
// stamped library is never the one bench.py times).  Every stamp is taken by the wave's first
// active lane, so a wave's time is counted once wherever it is (also inside divergent code):
// lap(i) adds the s_memtime cycles since the wave's previous lap to slot i; count(i) adds 1.
// Slots (tools/stamps.py): 0 refill, 1 walk: node visits, 2 walk: leaf rounds, 3 certificate +
// hit attributes, 4 hit shading, 5 rest of the loop (sky, pass bookkeeping, RayGen, write-back),
// 6 ray setup, 7 platforms; counts: 8 outer rounds, 9 walk iterations, 10 leaf rounds;
// 11 / 12: slots 1 / 2 in walk iterations with <= 8 working lanes (the tail), 13 their count.
// The block's per-wave slots live in LDS; flush() adds them to out[0..15].
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cpt {
namespace stamps {
constexpr int N_SLOTS = 16;   // slot 15: the wave's last stamp

#ifdef CPT_STAMPS
__device__ __forceinline__ unsigned long long* wave_slots() {
    __shared__ unsigned long long s[16 * N_SLOTS];   // up to 16 waves per block
    return s + (threadIdx.x >> 6) * N_SLOTS;
}
__device__ __forceinline__ bool first_active() {
    return (int)(threadIdx.x & 63) == __ffsll((unsigned long long)__ballot(1)) - 1;
}
__device__ __forceinline__ void init() {   // whole wave active
    if ((threadIdx.x & 63) < N_SLOTS) wave_slots()[threadIdx.x & 63] = 0;
    if ((threadIdx.x & 63) == 0) wave_slots()[N_SLOTS - 1] = __builtin_amdgcn_s_memtime();
}
__device__ __forceinline__ void lap(int i) {
    if (first_active()) {
        unsigned long long* s = wave_slots();
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        s[i] += t - s[N_SLOTS - 1];
        s[N_SLOTS - 1] = t;
    }
}
__device__ __forceinline__ void count(int i) {
    if (first_active()) wave_slots()[i] += 1;
}
__device__ __forceinline__ void flush(unsigned long long* out) {   // whole wave active
    if ((threadIdx.x & 63) < N_SLOTS - 1) atomicAdd(out + (threadIdx.x & 63), wave_slots()[threadIdx.x & 63]);
}
#else
__device__ __forceinline__ void init() {}
__device__ __forceinline__ void lap(int) {}
__device__ __forceinline__ void count(int) {}
__device__ __forceinline__ void flush(unsigned long long*) {}
#endif
}  // namespace stamps

// DIAGNOSTIC lane-occupancy timeline (CPT_TIMELINE builds only; never the timed library): at the
// top of every round of the megakernel each wave adds, for the time since its previous round
// (s_memrealtime, 100 MHz), busy lanes x dt and 64 x dt to the bin of the current time, and busy x
// dt again to a second / third slot when the wave has seen the pixel queue run dry / is a level-0
// (keeper) wave of the tail consolidation.  Bins of 2^TL_SHIFT ticks (1.31 ms) on a ring of
// TL_BINS (5.4 s); meta[0] = the first time a wave saw the queue dry (atomicMin).
// tools/timeline.py reads it through cpt_debug_timeline.
namespace timeline {
constexpr int TL_BINS = 4096, TL_SHIFT = 17, TL_WORDS = TL_BINS * 4 + 4;
// a wave's accumulators for the bin it is in (flushed to the global bins when the bin changes)
struct State {
    unsigned long long last, acc[4];
    uint32_t bin;
};
#ifdef CPT_TIMELINE
static __device__ unsigned long long g_tl[TL_WORDS];
__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ void init(State& st) {
    st.last = now();
    st.bin = (uint32_t)(st.last >> TL_SHIFT) & (uint32_t)(TL_BINS - 1);
    st.acc[0] = st.acc[1] = st.acc[2] = st.acc[3] = 0;
}
__device__ __forceinline__ void flush(State& st) {
    if ((int)(threadIdx.x & 63) == __ffsll((unsigned long long)__ballot(1)) - 1)
        for (int k = 0; k < 4; ++k)
            if (st.acc[k]) atomicAdd(&g_tl[4 * st.bin + k], st.acc[k]);
    st.acc[0] = st.acc[1] = st.acc[2] = st.acc[3] = 0;
}
__device__ __forceinline__ void round(State& st, uint64_t busy, bool exhausted, uint32_t level) {
    const unsigned long long t = now(), dt = t - st.last;
    st.last = t;
    const uint32_t b = (uint32_t)(t >> TL_SHIFT) & (uint32_t)(TL_BINS - 1);
    if (b != st.bin) {
        flush(st);
        st.bin = b;
    }
    const unsigned long long n = (unsigned long long)__popcll(busy);
    st.acc[0] += n * dt;
    st.acc[1] += 64ull * dt;
    if (exhausted) {
        if (st.acc[2] == 0 && (int)(threadIdx.x & 63) == __ffsll((unsigned long long)__ballot(1)) - 1)
            atomicMin(&g_tl[4 * TL_BINS], t);
        st.acc[2] += n * dt;
    }
    if (level == 0) st.acc[3] += n * dt;
}
#else
__device__ __forceinline__ unsigned long long now() { return 0; }
__device__ __forceinline__ void init(State&) {}
__device__ __forceinline__ void flush(State&) {}
__device__ __forceinline__ void round(State&, uint64_t, bool, uint32_t) {}
#endif
}  // namespace timeline

// DIAGNOSTIC exec-mask census (CPT_EXECDIAG builds only; never the timed library): lanes(out, r)
// records one entry of code region r by the wave with its active-lane count -- out[r] entries,
// out[16 + r] entries with <= 16 active lanes, out[32 + r] with <= 8, out[48 + r] the sum of
// active lanes -- by global atomics from the wave's first active lane.  With several waves per
// CU a VALU instruction with few active lanes costs several times the cycles of a full one
// (tools/exec_count_probe.hip), so a region entered thinly is a candidate for predication.
// Regions: tools/execdiag.py.
namespace execdiag {
constexpr int N_REGIONS = 16;
#ifdef CPT_EXECDIAG
__device__ __forceinline__ void lanes(unsigned long long* out, int r) {
    const uint64_t m = __ballot(1);
    if ((int)(threadIdx.x & 63) == __ffsll((unsigned long long)m) - 1) {
        const unsigned long long n = (unsigned long long)__popcll(m);
        atomicAdd(out + r, 1ull);
        if (n <= 16) atomicAdd(out + N_REGIONS + r, 1ull);
        if (n <= 8) atomicAdd(out + 2 * N_REGIONS + r, 1ull);
        atomicAdd(out + 3 * N_REGIONS + r, n);
    }
}
#else
__device__ __forceinline__ void lanes(unsigned long long*, int) {}
#endif
}  // namespace execdiag

// DIAGNOSTIC supply / demand of a cross-wave walk pool (CPT_POOLDIAG builds only; never the timed
// library; exclusive with CPT_EXECDIAG, whose counters it reuses): would the lanes of a wave that
// have finished their walk while others of the wave still walk find a suspended walk of another
// wave of the workgroup to continue?  A workgroup LDS count of the walks suspended right now
// (trace_wide returns 2 for them; they resume in their own wave's next round); in every node-visit
// iteration of the wide walk: idle = lanes of the call whose walk has ended, supply = that count.
// out[0] iterations, [1] sum idle, [2] sum min(idle, supply), [3] sum working lanes, [4] sum
// supply, [5] walks suspended, [6] walk calls (per wave).
namespace pooldiag {
#ifdef CPT_POOLDIAG
__device__ __forceinline__ uint32_t* susp() {
    __shared__ uint32_t s;
    return &s;
}
__device__ __forceinline__ unsigned long long* wave_acc() {
    __shared__ unsigned long long a[16 * 8];
    return a + (threadIdx.x >> 6) * 8;
}
__device__ __forceinline__ void init() {   // before the block's first barrier
    if (threadIdx.x == 0) *susp() = 0;
    if ((threadIdx.x & 63) < 8) wave_acc()[threadIdx.x & 63] = 0;
}
__device__ __forceinline__ bool leader() {
    return (int)(threadIdx.x & 63) == __ffsll((unsigned long long)__ballot(1)) - 1;
}
__device__ __forceinline__ void resumed(uint32_t n) {
    if (n && leader()) atomicSub(susp(), n);
    if (leader()) wave_acc()[6] += 1;
}
__device__ __forceinline__ void suspended(uint32_t n) {
    if (n && leader()) {
        atomicAdd(susp(), n);
        wave_acc()[5] += n;
    }
}
__device__ __forceinline__ void iteration(uint32_t idle, uint32_t working) {
    if (leader()) {
        const uint32_t sup = *(volatile uint32_t*)susp();
        unsigned long long* a = wave_acc();
        a[0] += 1;
        a[1] += idle;
        a[2] += idle < sup ? idle : sup;
        a[3] += working;
        a[4] += sup;
    }
}
__device__ __forceinline__ void flush(unsigned long long* out) {   // whole wave active
    if ((threadIdx.x & 63) < 8) atomicAdd(out + (threadIdx.x & 63), wave_acc()[threadIdx.x & 63]);
}
#else
__device__ __forceinline__ void init() {}
__device__ __forceinline__ void resumed(uint32_t) {}
__device__ __forceinline__ void suspended(uint32_t) {}
__device__ __forceinline__ void iteration(uint32_t, uint32_t) {}
__device__ __forceinline__ void flush(unsigned long long*) {}
#endif
}  // namespace pooldiag
}  // namespace cpt
