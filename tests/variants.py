"""Render-path selection for the bit-identity tests: every compiled kernel variant (the shipped ones and
the one A/B alternate, DF_ALT: the out-of-line drain lane groups) and drain / refill setting of both kernel
classes (rt_ctx_set_option; the library reads no environment)."""
import contextlib


def defaults(R):
    return {R.OPT_KERNEL: R.KERNEL_AUTO, R.OPT_VARIANT: -1, R.OPT_COOP: -1, R.OPT_COOP_MAX: 0, R.OPT_REFILL: 0,
            R.OPT_FAN: 1, R.OPT_INTERLEAVE: -1, R.OPT_FAN_CAP: 0, R.OPT_DUAL_STEP: -1, R.OPT_OPAQUE: -1,
            R.OPT_CENTRE_FIRST: -1, R.OPT_TREE: -1, R.OPT_INTERLEAVE_TAIL: 0, R.OPT_WAVEFRONT: -1, R.OPT_WF_BUILD: 0, R.OPT_WF_STREAMS: 0, R.OPT_PRIO: -1, R.OPT_WF_CHUNK: 0}


def kernel_classes(R):
    """The two shipped kernels, default variant each (textured and counting renders run these)."""
    return [{R.OPT_KERNEL: R.KERNEL_WHOLE_TRAVERSAL}, {R.OPT_KERNEL: R.KERNEL_DYNAMIC_FETCH}]


def all_variants(R):
    wt, df = R.KERNEL_WHOLE_TRAVERSAL, R.KERNEL_DYNAMIC_FETCH
    out = [{R.OPT_KERNEL: wt, R.OPT_VARIANT: v} for v in R.WT_VARIANTS]
    out += [{R.OPT_KERNEL: df, R.OPT_VARIANT: v} for v in R.DF_VARIANTS]
    out += [
        {R.OPT_KERNEL: df, R.OPT_COOP: 0},                      # no drain lane groups
        {R.OPT_KERNEL: df, R.OPT_COOP_MAX: 1},                  # drain groups of 64 lanes only
        {R.OPT_KERNEL: df, R.OPT_COOP: 2, R.OPT_REFILL: 64},    # full-wave refill + straggler groups
        {R.OPT_KERNEL: df, R.OPT_REFILL: 8},
        {R.OPT_KERNEL: df, R.OPT_FAN: 0},                       # spherical-light samples per lane
        {R.OPT_KERNEL: df, R.OPT_VARIANT: R.DF_BATCH, R.OPT_FAN: 0},
        {R.OPT_KERNEL: df, R.OPT_INTERLEAVE: 1, R.OPT_FAN: 0},  # a wave's pixels spread over 64 tiles
        {R.OPT_KERNEL: df, R.OPT_INTERLEAVE: 0},
        {R.OPT_KERNEL: df, R.OPT_CENTRE_FIRST: 1},              # upper-half tile ranges walked bottom-up
        {R.OPT_KERNEL: wt, R.OPT_INTERLEAVE: 1},
        {R.OPT_KERNEL: df, R.OPT_DUAL_STEP: 0},                 # one record or one node visit per step
        {R.OPT_KERNEL: df, R.OPT_VARIANT: R.DF_BATCH, R.OPT_DUAL_STEP: 0},
        {R.OPT_KERNEL: df, R.OPT_VARIANT: R.DF_ALT, R.OPT_COOP: 2, R.OPT_REFILL: 64},  # out-of-line drain, steady state
        {R.OPT_KERNEL: df, R.OPT_OPAQUE: 0},                    # general kernels where the opaque one is eligible
        {R.OPT_KERNEL: df, R.OPT_OPAQUE: 1},                    # the opaque kernel's 4-wave build without SPLIT
        {R.OPT_KERNEL: df, R.OPT_OPAQUE: 2},                    # ... its 3-wave build
        {R.OPT_KERNEL: df, R.OPT_OPAQUE: 3},                    # ... its 4-wave build with the re-visit group stack
        {R.OPT_KERNEL: df, R.OPT_OPAQUE: 4},                    # ... its 4-wave build, segments beside the mirror chain
        {R.OPT_KERNEL: df, R.OPT_OPAQUE: 5},                    # ... the same in the 3-wave build
        {R.OPT_KERNEL: df, R.OPT_OPAQUE: 7},                    # ... SPLIT without the drain lane groups
        {R.OPT_KERNEL: df, R.OPT_PRIO: 4},                      # ... issue priority after 4 iterations of a phase
        {R.OPT_KERNEL: df, R.OPT_REFILL: 32},                   # ... and a half-wave refill
        {R.OPT_KERNEL: df, R.OPT_COOP: 1},                      # ... drain lane groups in the drain only
        {R.OPT_KERNEL: df, R.OPT_TREE: 0},                      # general kernels where the tree kernel is eligible
        {R.OPT_KERNEL: df, R.OPT_TREE: 1},                      # the tree kernel with the re-visit group stack
        {R.OPT_KERNEL: df, R.OPT_TREE: 2},                      # ... and with the direct one (its default)
        {R.OPT_KERNEL: df, R.OPT_TREE: 3},                      # ... its 4-wave build with every index checked
        {R.OPT_KERNEL: df, R.OPT_TREE: 4},                      # ... its 4-wave build (view batches' default)
        {R.OPT_KERNEL: df, R.OPT_TREE: 5},                      # ... its 3-wave build (single frames' default)
        {R.OPT_KERNEL: df, R.OPT_WAVEFRONT: 0},                 # the opaque megakernel where the wavefront is eligible
        {R.OPT_KERNEL: df, R.OPT_WAVEFRONT: 1},                 # the wavefront path (trace / shade kernels)
        {R.OPT_KERNEL: df, R.OPT_WAVEFRONT: 2},                 # ... its trace kernel refilling at 2 waiting lanes
        {R.OPT_KERNEL: df, R.OPT_WAVEFRONT: 32},                # ... and at 32
        {R.OPT_KERNEL: df, R.OPT_WAVEFRONT: 1, R.OPT_WF_BUILD: 1},  # ... its trace kernel's 6-wave build
        {R.OPT_KERNEL: df, R.OPT_WAVEFRONT: 1, R.OPT_WF_BUILD: 2},  # ... 4 waves with the node prefetch
        {R.OPT_KERNEL: df, R.OPT_WAVEFRONT: 1, R.OPT_WF_BUILD: 3},  # ... 8 waves
        {R.OPT_KERNEL: df, R.OPT_WAVEFRONT: 1, R.OPT_WF_STREAMS: 3},  # ... its chunks over three streams
        {R.OPT_KERNEL: df, R.OPT_WAVEFRONT: 1, R.OPT_WF_BUILD: 4},  # ... node and record loads of a step together
        {R.OPT_KERNEL: df, R.OPT_WAVEFRONT: 1, R.OPT_WF_BUILD: 5},  # ... the same at 4 waves
        {R.OPT_KERNEL: df, R.OPT_WAVEFRONT: 1, R.OPT_WF_CHUNK: 128, R.OPT_WF_STREAMS: 3},  # ... 2-tile chunks (boundaries)
    ]
    return out


@contextlib.contextmanager
def options(R, ctx, opts):
    """Apply rt_ctx_set_option settings for the block, then restore the shipped defaults."""
    try:
        for k, v in opts.items():
            ctx.set_option(k, v)
        yield
    finally:
        for k, v in defaults(R).items():
            ctx.set_option(k, v)
