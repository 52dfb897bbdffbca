"""Execution policy of one network: the arithmetic its convs use, whether its
BN statistics are synchronised across ranks, and the measured tuning choices of
the kernel walk.  A policy is an immutable value carried by the model
(``KeypointsGauss.policy``) or passed explicitly to ``hkp.net`` — the product
keeps no process-global switches and reads no environment variables, so two
models (or two threads) with different policies never interfere.

Tuning fields hold the measured defaults; A/B tooling builds
non-default policies explicitly (``tools/knobs.py``, ``bench.py --tune``).
"""
from dataclasses import dataclass, fields, replace

# Conv arithmetic of the NHWC convs and the stem:
#   "fp32"  v_mfma_f32_32x32x2_f32, exact fp32 products
#   "f16x3" split-precision fp16 MFMA, fp32-accurate (~2^-22 per product)
#   "f16"   plain fp16 operands and activations, fp32 accumulation (BASELINE
#           config C4, inference): one fp16 MFMA per MAC, fp16 conv outputs and
#           residual stream (autocast semantics)
#   "f16x2w" / "f16x2a"  inference modes between the two (DESIGN "precision
#           modes"): the f16x3 data path (packed split activations, fp32 conv
#           outputs and BN) with two of the three fp16 products per MAC — the
#           weights ("w") or the conv's input activation ("a") rounded to fp16
# value: the operand layout the producers emit (3 packed split, 1 plain fp16, 0 fp32)
PRECISIONS = {"fp32": 0, "f16x3": 3, "f16": 1, "f16x2w": 3, "f16x2a": 3}
# hkp_conv2d_fwd_x3_products product set of each packed-split precision
PRODUCTS = {"f16x3": 3, "f16x2w": 2, "f16x2a": 4}
INFERENCE_ONLY = ("f16", "f16x2w", "f16x2a")


@dataclass(frozen=True)
class Policy:
    precision: str = "f16x3"
    # SyncBN (caveat D5): train-mode BN statistics and their backward
    # sums over every rank of `sync_group` (None = the default world group)
    sync_bn: bool = False
    sync_group: object = None
    # --- tuning (measured defaults) ----------------------------------------
    # a conv's wgrad runs on a side stream concurrently with its dgrad
    overlap_wgrad: bool = True
    # ... only for convs of at least this many GFLOP per pass (2*M*K*C*R*S): below
    # it the wgrad's one-block-per-CU grid holds the whole GPU while the dgrad
    # waits, and the cross-stream join costs more than the overlap saves
    overlap_min_gflop: float = 0.0
    # HKP_TILE_* of a dgrad overlapped by its wgrad: 11 = the A3 256x256 body, its
    # last partial round as whole tiles (in-process A/B on the C3 shard, 7 rounds:
    # 464.3 img/s vs 460.9 for 9 = 2-stage 256x256 + split-K tail launch, 453.0 for
    # the planner)
    dgrad_overlap_tile: int = 11
    # ... with the split-K workspace (the A3 grid's last partial round as split-K
    # segments inside the same launch, stream-K plans for the 64/128-wide dgrads):
    # measured +0.5 % in round 4, but beside the halo wgrads and the CU budgets
    # below, without it: 487.7 vs 484.8 and 489.0 vs 485.7 img/s (in-process A/Bs,
    # 11 / 7 rounds, profiles/r06_gapsk_ab.log, r06_wgh_ab_train_dgsk.log)
    dgrad_overlap_sk: bool = False
    # CUs a wgrad overlapped by its dgrad spreads its pixel-range splits over
    # (0 = the planner's split count, filling every CU as if it ran alone)
    wgrad_overlap_cus: int = 192
    # the halo wgrad body for the 3x3 stride-1 convs of <= 128 channels (the
    # library's planner choice); False keeps the tiled body (A/B)
    wgrad_halo: bool = True
    # ... and the CUs an overlapped halo wgrad spreads its pixel ranges over (0:
    # wgrad_overlap_cus): fewer than all leave CUs to the dgrad it overlaps.  C3
    # shard, in-process A/B, 9 rounds: 488.3 img/s (192 / 160) vs 481.8 for the
    # tiled body at 0 / 0 and 485.9 for 192 / 192 (profiles/r06_wgh_ab_train_cus5.log);
    # C5 77.4 vs 77.0 (halo vs tiled; the budgets neutral there)
    wgrad_halo_cus: int = 160
    # inner BN ReLU masks recomputed from y in the backward (no fp32 activation kept)
    mask_from_y: bool = True
    # inference: last block's BN apply fused with the K-row head
    fused_head: bool = True
    # HKP_TILE_* of the plain-fp16 1x1 / kxk convs and of the f16x3 forward convs
    # (0 = the planner)
    f16_tile_1x1: int = 0
    f16_tile_kxk: int = 0
    # the Bottleneck's conv3 with bn3 + residual + ReLU in its epilogue (C4); -1 =
    # f16_tile_1x1
    f16_tile_fused: int = -1
    x3_tile: int = 0
    # training: repeat the last batched weight-pack launch when it repacks every operand
    prepack_plan: bool = True
    # BN finalize: two-level merge from this many partial tiles on
    fin_two_level_tiles: int = 2048
    # plain fp16 inference (C4): a Bottleneck's bn3 statistics from conv3's input
    # covariance (1x1 conv: exact), bn3 + residual + ReLU in conv3's epilogue
    gram_bn: bool = True
    # inference: a block's inner BN + ReLU applied inside the next conv where that
    # conv runs the halo-tile body (hkp_conv2d_fwd_x3_bnin / _f16_bnin: layer1's
    # 3x3 convs at 640x480) instead of a separate apply pass
    fuse_input_bn: bool = True
    # forward conv tiles from the measured plan table (hkp/tile_plan.json, written by
    # tools/tile_sweep.py) where it holds the conv's shape; the C planner elsewhere
    # (a nonzero x3_tile / f16_tile_* field still forces its policy)
    tile_plan: bool = True
    # inference, per-stage conv arithmetic (DESIGN "Per-stage precision"): () = every
    # stage at `precision`; else one of "f16" / "f16x3" for each of layer1..layer4
    # (the stem conv is fp32-class in both; the head follows layer4), the
    # activation converted where two stages meet
    stage_precision: tuple = ()

    def __post_init__(self):
        if self.precision not in PRECISIONS:
            raise ValueError("precision must be one of %s, got %r" % (sorted(PRECISIONS), self.precision))
        if self.stage_precision and (len(self.stage_precision) != 4 or
                                     any(p not in ("f16", "f16x3") for p in self.stage_precision)):
            raise ValueError("stage_precision: four of 'f16' / 'f16x3' (layer1..layer4), got %r"
                             % (self.stage_precision,))

    @property
    def passes(self):
        return PRECISIONS[self.precision]

    @property
    def products(self):
        """hkp_conv2d_fwd_x3_products product set of the packed-split forward convs."""
        return PRODUCTS.get(self.precision, 3)

    def with_(self, **kw):
        return replace(self, **kw)


DEFAULT = Policy()

TUNING_FIELDS = tuple(f.name for f in fields(Policy) if f.name not in ("precision", "sync_bn", "sync_group",
                                                                      "stage_precision"))


def resolve(policy):
    return DEFAULT if policy is None else policy
