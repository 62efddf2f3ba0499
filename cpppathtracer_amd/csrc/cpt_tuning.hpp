// cpt_tuning.hpp — the megakernel's scheduling constants, in one place.  Each value was chosen by
// interleaved same-box A/Bs (DESIGN.md §Tuning record; logs under profiles/); none changes a
// result, only which lanes work together when.
#pragma once

namespace cpt {

// Persistent LDS-walk workgroup: 1024 lanes = 16 waves, 4 per SIMD (the tree image, the 16-bit
// walk stacks and the pending sky fetches take 156 KB of the CU's 160 KB; 128 VGPRs).
// 768 lanes (3 waves/SIMD): 1153 vs 1256 Mpaths/s (profiles/r02/ab_w4_1024.log); r05 re-check 1759
// vs 1930-1974 (profiles/r05/ab_lds_block_768.log).
constexpr int LDS_BLOCK = 1024;
// Occupancy target of the kernels without the LDS tree image (reference and binary walks).
constexpr int WAVES_PER_SIMD = 3;
// A round's walks are suspended once at most SUSPEND_AT lanes of the wave still walk and at least
// SUSPEND_MIN_DONE lanes of the call have finished theirs (cpt_path.hpp trace_wide):
// 1356-1392 vs 1304 Mpaths/s without suspension (profiles/r02/ab_suspend*.log, ab_threshold_combo.log).
constexpr int SUSPEND_AT = 8;
constexpr int SUSPEND_MIN_DONE = 40;
// Leaf rounds of the wide walk run when this many 64ths of the wave's working lanes are stopped
// at a parked leaf (profiles/r01n_ab_thresholds_resweep.log, r02/ab_threshold_combo.log).
constexpr int SPEC_LEAF_ROUND = 28;
// Deferred sky fetches run when this many 64ths of the tracing lanes hold one
// (profiles/r01l_ab_defer_miss.log, r02/ab_threshold_combo.log).
constexpr int DEFER_MISS_ROUND = 40;
// With the cost schedule, each wave's first tile is placed by consolidation level (the heaviest
// tiles to the level-0 wave of every SIMD) instead of taken from the counter
// (profiles/r02/reh_static_first_*.log; r05: C4 neutral, C2 30.2k vs 24.0k Mpaths/s without it).
constexpr bool STATIC_FIRST = true;
// The refill draws a tile's worth of pixel ids per counter atomic and serves the wave's idle lanes
// from them over the following rounds (cpt_kernels.hip k_megakernel).  1-spp C4 render 1.43 vs
// 2.43 ms; 128 ids 1.50 ms; requesting the next range ahead of need 1.49-1.56 ms
// (profiles/r04/ab_take_batch_*.log); 32 / 128 ids for long chains tied / lost (r05
// ab_take_range_long.log).  The consolidating kernel takes exactly what it needs: its ranks hold
// <= 4 pixels per lane, and ranges of 4 / 8 / 16 / 64 ids, the taper and a workgroup-shared range
// all lost there (r04 ab_take_hold_rehearsal.log, ab_take_workgroup.log; r05 reh_cons_take_sizes.log,
// reh_cons_taper.log).
constexpr int TAKE_BATCH = 64;
// Long chains: the range a wave draws shrinks as 64 x left / (TAKE_TAPER x grid lanes) (guided
// scheduling), so the ids waves hold unstarted stay below 1/TAKE_TAPER of a lane-round.  r05
// (profiles/r05/ab_take_*.log), C2 / C4: no taper 24.4k / 1982; taper 2 29.5k / 1965; taper 4
// 30.1k / 1982; taper 8 30.4k / 1952 Mpaths/s.
constexpr int TAKE_TAPER = 4;
// Tail consolidation: a level-L wave (L = 1..3) retires, handing its chains to the keepers, once the
// workgroup's live chains are at most L x this (each retiring wave hands over <= 64 chains, so the
// slab's 3 x 256 slots hold every hand-over whatever the value).  r05 rehearsal, C5 N = 8 slowest
// rank (profiles/r05/reh_cons_retire_threshold.log): 128 / 192 / 384 2574-2582 ms against 2521 /
// 2551 at 256.
constexpr int CONS_RETIRE_PER_LEVEL = 256;

}  // namespace cpt
