// cpt_tuning.hpp — the megakernel's scheduling constants, in one place.  Each value was chosen by
// interleaved same-box A/Bs at C4 (the A/B tables; logs under profiles/); none changes
// a result, only which lanes work together when.  The #ifndef lets an A/B build
// (cpppathtracer_amd/build.py defines=...) override one; the shipped library uses these values.
#pragma once

namespace cpt {

// Persistent LDS-walk workgroup: 1024 lanes = 16 waves, 4 per SIMD (the tree image, the 16-bit
// walk stacks and the pending sky fetches take 156 KB of the CU's 160 KB; 128 VGPRs).
// 768 lanes (3 waves/SIMD): 1153 vs 1256 Mpaths/s (profiles/r02/ab_w4_1024.log).
#ifndef CPT_LDS_BLOCK
#define CPT_LDS_BLOCK 1024
#endif
// Occupancy target of the kernels without the LDS tree image (reference and binary walks).
#ifndef CPT_WAVES_PER_SIMD
#define CPT_WAVES_PER_SIMD 3
#endif
// A round's walks are suspended once at most this many lanes of the wave still walk and at
// least SUSPEND_MIN_DONE lanes of the call have finished theirs (cpt_path.hpp trace_wide):
// 1356-1392 vs 1304 Mpaths/s without suspension (profiles/r02/ab_suspend*.log, ab_threshold_combo.log).
#ifndef CPT_SUSPEND_AT
#define CPT_SUSPEND_AT 8
#endif
#ifndef CPT_SUSPEND_MIN_DONE
#define CPT_SUSPEND_MIN_DONE 40
#endif
// Leaf rounds of the wide walk run when this many 64ths of the wave's working lanes are stopped
// at a parked leaf (profiles/r01n_ab_thresholds_resweep.log, r02/ab_threshold_combo.log).
#ifndef CPT_SPEC_LEAF_ROUND
#define CPT_SPEC_LEAF_ROUND 28
#endif
// Deferred sky fetches run when this many 64ths of the tracing lanes hold one
// (profiles/r01l_ab_defer_miss.log, r02/ab_threshold_combo.log).
#ifndef CPT_DEFER_MISS_ROUND
#define CPT_DEFER_MISS_ROUND 40
#endif
// With the cost schedule, each wave's first tile is placed by consolidation level (the heaviest
// tiles to the level-0 wave of every SIMD) instead of taken from the counter
// (profiles/r02/reh_static_first_*.log).  Round 5 (profiles/r05/ab_static_first.log): C4 neutral
// (1969-1990 vs 1976-2000), C2 30.2k vs 24.0k Mpaths/s without it.
#ifndef CPT_STATIC_FIRST
#define CPT_STATIC_FIRST 1
#endif

// The refill draws a tile's worth of pixel ids (64) per counter atomic and serves the wave's
// idle lanes from them over the following rounds (cpt_kernels.hip k_megakernel; 0 = one atomic
// per refill).  1-spp C4 render 1.43 vs 2.43 ms; 128 ids 1.50 ms; requesting the next range
// ahead of need 1.49-1.56 ms and up to 10% slower at 1024 spp (profiles/r04/ab_take_batch_*.log).
#ifndef CPT_TAKE_BATCH
#define CPT_TAKE_BATCH 64
#endif
// Long chains (spp >= 64) take ranges of CPT_TAKE_BATCH_LONG ids.  The consolidating kernel
// (frames of <= 4 pixels per lane, the strong-scaling ranks) takes exactly what it needs unless
// CPT_TAKE_BATCH_CONS: there a wave's unstarted ids are a large share of the frame's work and
// hold back long chains other waves' idle lanes could run (C4 rehearsal N = 2 / 4: 677 / 469 ms
// batched vs 622 / 416 exact; C5 N = 8 2787 vs 2528; profiles/r04/ab_take_hold_rehearsal.log).
#ifndef CPT_TAKE_BATCH_LONG
#define CPT_TAKE_BATCH_LONG 64
#endif
#ifndef CPT_TAKE_BATCH_CONS
#define CPT_TAKE_BATCH_CONS 0
#endif
// The consolidating kernel's range size when CPT_TAKE_BATCH_CONS is set.  Round 5, C5 N = 8
// rehearsal (slowest rank, two interleaved rounds; exact takes 2542 / 2590 ms): 4 ids 2635 / 2597,
// 8 ids 2618 / 2582, 16 ids 2682 / 2622 (profiles/r05/reh_cons_take_sizes.log).  Exact stays.
#ifndef CPT_TAKE_BATCH_CONS_SIZE
#define CPT_TAKE_BATCH_CONS_SIZE 64
#endif
// Long chains: the leader reads the pixel counter before sizing a draw, so the range size sees
// the counter's current value rather than the wave's last draw (advisor r04).  2: only until
// the wave's last draw left less than one id per lane of the grid (the tail, where draws are
// frequent and nearly exact anyway); 1: on every draw.
#ifndef CPT_TAKE_FRESH
#define CPT_TAKE_FRESH 2
#endif
// Long chains: the range a wave draws shrinks as 64 x left / (TAPER x grid lanes) (guided
// scheduling), so the ids waves hold unstarted stay below 1/TAPER of a lane-round.  0: full
// ranges until one id per lane is left, then exact draws — then up to a whole lane-round of ids
// sits in waves' ranges when the tail starts, a chain-time lost at frames of few pixels per lane.
// Round 5 (profiles/r05/ab_take_*.log), C2 (3.5 pixels per lane) / C4 (7.9): taper 0 with
// fresh 1 24.4k / 1982; fresh 2 28.8k / 1963; taper 2 29.5k / 1965; taper 4 30.1k / 1982;
// taper 8 30.4k / 1952; one atomic per take (CPT_TAKE_BATCH 0) 30.7k / 1954 Mpaths/s.
#ifndef CPT_TAKE_TAPER
#define CPT_TAKE_TAPER 4
#endif

// Tail consolidation: a level-L wave (L = 1..3) retires, handing its chains to the keepers, once
// the workgroup's live chains are at most L x this (each retiring wave hands over <= 64 chains, so
// the slab's 3 x 256 slots hold every hand-over whatever the value).  Round 5 rehearsal, C5 N = 8
// slowest rank (profiles/r05/reh_cons_retire_threshold.log): 128 / 192 / 384 2574-2582 ms against
// 2521 / 2551 at 256; 384 also costs C4 N = 8 (380 vs 322 ms).
#ifndef CPT_CONS_RETIRE_PER_LEVEL
#define CPT_CONS_RETIRE_PER_LEVEL 256
#endif

// The LDS kernels' cold walks out of line (cpt_path.hpp trace_cold).
#ifndef CPT_COLD_NOINLINE
#define CPT_COLD_NOINLINE 0
#endif

constexpr int SUSPEND_AT = CPT_SUSPEND_AT;
constexpr int SUSPEND_MIN_DONE = CPT_SUSPEND_MIN_DONE;
constexpr int SPEC_LEAF_ROUND = CPT_SPEC_LEAF_ROUND;
constexpr int DEFER_MISS_ROUND = CPT_DEFER_MISS_ROUND;
constexpr bool STATIC_FIRST = CPT_STATIC_FIRST != 0;

}  // namespace cpt
