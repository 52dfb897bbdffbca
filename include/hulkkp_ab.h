/*
 * hulkkp_ab.h — A/B instruments of the tools-only build of libhulkkp
 * (`make -C hulk-keypoints_amd/csrc ab` -> tools/ab_lib/libhulkkp_ab.so, compiled
 * with -DHKP_AB_KNOBS).  The product library (include/hulkkp.h) does not export
 * these: it compiles every knob below as a constant at its default and keeps no
 * process-global switches.  Every setter is process-global and not thread-safe;
 * tools/ set them in one thread, around their own measurements.
 */
#ifndef HULKKP_AB_H
#define HULKKP_AB_H

#include "hulkkp.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Debug (tools/ only, not thread-safe): one-tile forward conv launches record
 * per-block phase clocks (s_memrealtime, 100 MHz) into buf[block * 8 + slot]
 * (start, pipeline filled, K loop done, BN partials done, output staged, stores
 * issued); NULL turns it off. */
void hkp_debug_x3_stamps(uint64_t* buf);
/* Debug / tuning (tools/ only, not thread-safe): one-tile forward conv launches
 * hold half the CUs of every XCD back for ns nanoseconds in their first round of
 * blocks (0 = off), so the rounds' epilogues do not all coincide. */
void hkp_debug_x3_stagger(int32_t ns);
/* Debug / A/B (tools/ only, not thread-safe): nonzero runs an A3 grid's split-K
 * tail as a launch of its own (conv_x3_tail_kernel) instead of appended to it. */
void hkp_debug_x3_split_tail(int32_t on);
/* Debug / A/B (tools/ only, not thread-safe): the flavour of the forward convs'
 * epilogue output stores: 0 each site's own (the default), 1 plain, 2
 * nontemporal, 3 sc1 (written through, not kept in the XCD's L2), 4 sc0 sc1. */
void hkp_debug_x3_store(int32_t kind);
/* Debug / A/B (tools/ only, not thread-safe): the DUO body's (HKP_TILE_DUO)
 * first-round delay of the second block on each CU, in ns (0 = off, < 0 = the
 * default estimate of half a block's lifetime). */
void hkp_debug_duo_stagger(int32_t ns);
/* Debug / A/B (tools/ only, not thread-safe): static wave priority in the A3 body's
 * K loop: 0 none (default), 1 s_setprio 1 on waves 4-7, 2 on waves 0-3. */
void hkp_debug_x3_prio(int32_t mode);
/* Debug / A/B (tools/ only, not thread-safe): nonzero runs the stem on the one-tile
 * kernel (as HKP_TILE_64_PAIR does per call) instead of the patch body. */
void hkp_debug_stem_pair(int32_t on);
/* Debug / A/B (tools/ only, not thread-safe): 0 returns AUTO's packed-f16x3 plans
 * to the round-4 cost table's: no 256x64 two-blocks-per-CU tiles for short-K convs
 * and 256x128 grids of >= 1 round, 32x32x16 MFMAs for one-round 256x128 grids. */
void hkp_debug_x3_pair128(int32_t on);
/* Debug / A/B (tools/ only, not thread-safe): 0 runs the BN finalize merges
 * (forward and backward) as batched-load loops where the default holds a tile
 * lane's partials in registers after one load round — the same bits either way. */
void hkp_debug_fin_regs(int32_t on);
/* A/B probe (tools/ only, not thread-safe): the one-tile conv bodies read the A
 * operand of output row m from row m % rows (0 = off): the outputs are wrong, the
 * activation stream L2-resident — times a conv's K loop without the HBM / MALL
 * latency of its activation lines (tools/conv_ab.py --a-wrap). */
void hkp_debug_x3_a_wrap(int32_t rows);

#ifdef __cplusplus
}
#endif
#endif
