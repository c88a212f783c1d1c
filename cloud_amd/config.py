"""The ``CLOUD_AMD_*`` environment namespace in one place.

Every switch the framework reads is declared here with its type, default and
meaning; ``get(name)`` parses it.  ``python -m cloud_amd.config`` prints the
table.  A test (``tests/test_config_env.py``) fails if code reads a
``CLOUD_AMD_*`` variable that is not declared here.  The reference-compatible
variables (``TF_CONFIG``, ``TF_KERAS_RUNNING_REMOTELY``) keep their names.
"""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass(frozen=True)
class Var:
    name: str
    type: type
    default: object
    doc: str
    area: str


_VARS = [
    # launcher / run()
    Var("CLOUD_AMD_JOBS_DIR", str, "./jobs", "where run() stages job directories", "launcher"),
    Var("CLOUD_AMD_HOME", str, "~/.cloud_amd", "per-user state: the job-id index (jobs/<id> -> job directory) that "
        "python -m cloud_amd.jobs uses to find a job from any directory", "launcher"),
    Var("CLOUD_AMD_STAGE_COPY", bool, False, "stage code files by copying too (default: code "
        "hard-linked, every other file copied; a running job then never sees in-place edits of its sources)", "launcher"),
    Var("CLOUD_AMD_CPU_AFFINITY", bool, True, "launcher pins each GPU rank to the cores of its GPU's NUMA node "
        "(KFD io_links + sysfs cpulist), split between the ranks on that node; 0 = leave placement to the OS",
        "launcher"),
    Var("CLOUD_AMD_NUMA_ROOT", str, "/sys/devices/system/node", "sysfs NUMA-node tree read for rank CPU placement "
        "(tests point it at a fake tree)", "launcher"),
    Var("CLOUD_AMD_CPU_ROOT", str, "/sys/devices/system/cpu", "sysfs CPU tree (SMT siblings) read for rank CPU "
        "placement (tests point it at a fake tree)", "launcher"),
    Var("CLOUD_AMD_NUM_GPUS", int, None, "override the visible-GPU count (0 = CPU node)", "launcher"),
    Var("CLOUD_AMD_RUNNING_REMOTELY", str, "", "set by the launcher inside job ranks (remote() is True)", "launcher"),
    Var("CLOUD_AMD_JOB_ID", str, "", "job id (set in every rank)", "launcher"),
    Var("CLOUD_AMD_JOB_DIR", str, "", "job directory (set in every rank)", "launcher"),
    Var("CLOUD_AMD_LAUNCH_TIME", float, None, "launcher spawn time, epoch seconds (set in every rank)", "launcher"),
    Var("CLOUD_AMD_RANK_T0", float, None, "wall time at which a launched rank's wrapper started (set by the "
        "generated entry-point wrapper; the benches split run()->first step into phases with it)", "launcher"),
    Var("CLOUD_AMD_RUN_T0", float, None, "run() entry time, for run()->first-step latency (set in ranks)",
        "launcher"),
    Var("CLOUD_AMD_PIP_INSTALL", bool, False, "pip install --user the job's requirements (needs an index)",
        "launcher"),
    Var("CLOUD_AMD_REGION", str, "local", "region string reported by topology.get_region()", "launcher"),
    Var("CLOUD_AMD_PROJECT", str, "local", "project name reported to the tuner / cloud_fit", "launcher"),
    Var("CLOUD_AMD_DEVICE", str, None, "force the strategy device (e.g. 'cpu')", "launcher"),
    Var("CLOUD_AMD_PG_TIMEOUT_S", float, 600.0, "torch.distributed process-group timeout", "launcher"),
    # kernels / ops
    Var("CLOUD_AMD_OPS", str, "native", "'native' HIP kernels or 'torch' stock ops", "ops"),
    Var("CLOUD_AMD_AUTOGRAD_MT", bool, False, "keep autograd's per-device backward worker thread (torch's default); "
        "off: backward runs on the calling thread, 1.3 ms less host time per BERT step (runtime/host.py)", "runtime"),
    Var("CLOUD_AMD_DETERMINISTIC", bool, False, "raise instead of taking an order-dependent float-atomic kernel "
        "path (embedding gradient with more than two token types or rows wider than the owner kernel holds)",
        "ops"),
    Var("CLOUD_AMD_GEMM", str, "native", "dense GEMMs: 'native' or 'torch'", "ops"),
    Var("CLOUD_AMD_CONV", str, "native", "convolutions: 'native' or 'torch'", "ops"),
    Var("CLOUD_AMD_GEMM_CORE", str, "auto", "GEMM core: 'auto' (128x128 LDS-DMA core plus the 256x256 two-phase "
        "core of ca_gemm256p8.h for large GEMMs), 'glds_ring' (128 core plus the 256x256 ring core), 'glds' (128 "
        "core only), 'vp8' / 'v256' (the two-phase / ring 256 core whenever M, N >= 256), 'glds8', 'reg' "
        "(register staging); 'glds_ring' / 'v256' / 'glds8' need CLOUD_AMD_BUILD_EXPERIMENTAL=1", "ops"),
    Var("CLOUD_AMD_BUILD_EXPERIMENTAL", bool, False, "build: also compile the experiment-only GEMM cores (glds8, "
        "256x256 ring, stream-K, 256x128) into _C for A/B runs", "ops"),
    Var("CLOUD_AMD_WGRAD_BLOCKS", int, 512, "convolution weight gradients: split-K so that about this many "
        "workgroups run (tiles x splits); fewer splits = less fp32 slab traffic, more = fuller CUs", "ops"),
    Var("CLOUD_AMD_WGRAD_BLOCKS_SMALLM", int, 512, "convolution weight gradients with <= 128 output channels "
        "(ResNet stem, layers 1-2): split-K workgroup target", "ops"),
    Var("CLOUD_AMD_STEM_WGRAD_BLOCKS", int, 2048, "space-to-depth stem weight gradient (the last kernel of the "
        "backward pass): split-K workgroup target", "ops"),
    Var("CLOUD_AMD_DENSE_WGRAD_BLOCKS", int, 640, "dense-layer weight gradients (BERT): split-K workgroup target "
        "(round 4, same box: 640 -> 6,993 / 6,993 seq/s, 768 -> 6,962 / 6,952, 1024 -> 6,892 / 6,911, 512 -> "
        "6,865 / 6,896; profiles/r4_s36/)",
        "ops"),
    Var("CLOUD_AMD_GEMM_256X128", bool, False, "GEMMs whose 256 x 128 grid fills whole rounds (and 256 x 256 does "
        "not) on the 256 x 128 single-phase core (csrc/include/ca_gemm256p8.h); measured slower than the 128 core "
        "on BERT's shapes", "ops"),
    Var("CLOUD_AMD_DENSE_WGRAD_256", bool, False, "dense-layer weight gradients whose 256 x 256 tiles times a split "
        "count fill one round of the chip (BERT QKV / FFN) run on the two-phase 256 core with that split (measured "
        "3 % slower on BERT than the 128 core's 1024-workgroup split: 6,749 / 6,754 vs 6,952 / 6,940 seq/s)", "ops"),
    Var("CLOUD_AMD_TAPMASK", bool, True, "convolutions: tap-mask / incremental buffer-mode gather loaders; 0 keeps "
        "the general per-chunk decode loaders (A/B runs)", "ops"),
    Var("CLOUD_AMD_SPLIT_XCD", bool, True, "split-K GEMM/conv grids: give each XCD contiguous (split, tile) "
        "ranges so the tiles of one K chunk share an L2; 0 remaps tiles only (A/B runs)", "ops"),
    Var("CLOUD_AMD_BN_APPLY_BLOCKS", int, 0, "BatchNorm apply passes (fwd y/mask, bwd dz): total workgroups of "
        "the HBM stream; 0 = the reduction kernels' tiling", "ops"),
    Var("CLOUD_AMD_BN_APPLY_ILV", bool, True, "BatchNorm apply passes: 1 = RP-row groups dealt round-robin to "
        "the workgroups (one contiguous sweep); 0 = one contiguous row chunk per workgroup", "ops"),
    Var("CLOUD_AMD_CONV_TALL", bool, True, "<= 64-channel 3x3 convolutions (fwd, stride-1 dgrad): 256 x 64 tiles "
        "with 4 x 1 waves; 0 = 128 x 64 with 2 x 2 waves", "ops"),
    Var("CLOUD_AMD_STEM_LDS", bool, True, "space-to-depth stem convolution forward on the LDS-resident patch + filter "
        "kernel (csrc/include/ca_conv_stem.h); 0 = the implicit-GEMM row-segment loader", "ops"),
    Var("CLOUD_AMD_STEM_TALL", bool, True, "space-to-depth stem convolution on the tall 256 x 64 tiles too (0.88 -> "
        "0.72 ms per call at b1024); 0 = 128 x 64 tiles (A/B runs)", "ops"),
    Var("CLOUD_AMD_STEM_BWD_RECOMPUTE", bool, True, "ResNet stem tail backward: a statistics-only max-pool "
        "backward pass, then the BN-backward apply recomputes the pooled gradient per 2x2 block (the 112x112 "
        "gradient is never written: 3.3 GB fewer per step at b1024).  With the window loads issued ahead of "
        "any branch: 0.65 + 0.90 ms against 1.09 + 0.94 for write-then-apply, +0.8 % end to end "
        "(profiles/r4_s44/); 0 = write g and run the separate apply pass", "ops"),
    Var("CLOUD_AMD_BN_GROUPS_MAX", int, 512, "BatchNorm statistics: most groups of the first-level reduction of the "
        "per-tile partial rows (1..512; ~64 rows per group)", "ops"),
    Var("CLOUD_AMD_GEMM_LIB", str, "never", "plain bf16 GEMMs (bias / accumulate only, no fused epilogue): 'never' "
        "(default: every GEMM on the in-tree kernels, the same engine on every box and rank), 'auto' (diagnostic: "
        "times the in-tree kernel against hipBLASLt once per shape and keeps the faster), 'always' "
        "(ops/raw.py PlainGemmPolicy)", "ops"),
    Var("CLOUD_AMD_GEMM_PRW", bool, True, "forward 1x1 convolutions with N = 256, K = 64 (ResNet layer-1 conv3 "
        "and shortcut): persistent resident-weight core (csrc/include/ca_gemm_prw.h); 0 = the tiled 128 core",
        "ops"),
    Var("CLOUD_AMD_GEMM_PRWN", bool, True, "forward 1x1 convolutions N = 512 / K = 128 and N = 1024 / K = 256 with "
        "BN statistics (ResNet stage-2 / stage-3 conv3): the persistent core with the weight resident in column "
        "chunks (ca_gemm_prw.h); 0 = the tiled 128 core", "ops"),
    Var("CLOUD_AMD_SMALLK_SET", str, "", "bench/smallk_gemm.py shape set ('conv3': the conv3 expansions of "
        "stages 2-4)", "bench"),
    Var("CLOUD_AMD_EPI_PF", bool, True, "GEMM epilogues that read memory or run an activation (BN-statistics "
        "forward 1x1 convs, BERT bias/GELU/GELU'/beta dense layers): 4 staged output rows in flight per trip", "ops"),
    Var("CLOUD_AMD_ATTN_FUSED_BWD", bool, True, "attention at S = 64 / 128: one workgroup per (batch, head) for "
        "the forward and a single fused backward kernel; 0 keeps the 64-query-block kernels", "ops"),
    Var("CLOUD_AMD_CONV_HALO_WGRAD", bool, True, "the weight gradient of the same 3x3 / 64-channel / width-56 "
        "convolutions on the LDS-resident kernel (ca_conv_halo.h conv3x3_halo_wgrad: 64 x 576 partial in registers, "
        "one fp32 slab per workgroup); 0 = implicit GEMM (A/B)", "ops"),
    Var("CLOUD_AMD_LN_BWD16", bool, False, "LayerNorm backward on 16-wave blocks, one row per wave, the block's "
        "partials summed by a fixed LDS tree (measured 2.8 % slower on BERT beside the weight-gradient side stream; "
        "default: 4-wave blocks walking four rows per wave)", "ops"),
    Var("CLOUD_AMD_GEMM_256X96", bool, True, "forward GEMMs whose 256 x 96 grid fills whole rounds while the 128 x "
        "128 grid leaves a partial one (BERT QKV, M = 8192, N = 2304) run on 256 x 96 tiles; 0 = off (A/B)", "ops"),
    Var("CLOUD_AMD_GEMM_STREAMK", int, 0, "two-phase 256 x 256 GEMM: 0 off (default; measured slower than the "
        "128 x 128 core on BERT's M = 8192 shapes), 1 stream-K on under-filled grids, 2 wherever allowed (tests)", "ops"),
    Var("CLOUD_AMD_LN_BWD8", bool, False, "retired round-5 A/B knob (8-wave LayerNorm backward, measured 1.5 % slower "
        "and removed); ignored", "ops"),
    Var("CLOUD_AMD_BN_FIN_RPG", int, 512, "BatchNorm statistics finalize: partial rows per group block (64-512)", "ops"),
    Var("CLOUD_AMD_BN_FIN_MERGED", bool, True, "BatchNorm statistics from many partial rows: group reduction and "
        "per-channel finalize in ONE launch (last block per 64 channels finalizes, agent-scope ticket); 0 = two "
        "launches (A/B runs)", "ops"),
    Var("CLOUD_AMD_CONV_HALO", int, 1, "3x3 / stride-1 / 64-channel convolutions at width 56 (ResNet-50 "
        "stage 1) forward and input gradient on the LDS-resident kernel (ca_conv_halo.h: input patch and all 9 taps "
        "in LDS, persistent grid); 0 = implicit-GEMM tiles, 2 = halo kernel without the software-pipelined "
        "fragment reads (A/B runs)", "ops"),
    Var("CLOUD_AMD_CONV_EPI_PF", bool, True, "implicit-GEMM forward convolutions with the BN-statistics epilogue: "
        "read 2 staged output rows from LDS before storing", "ops"),
    Var("CLOUD_AMD_SHAPE_LOG", str, None, "profiling: append one JSON line per GEMM/convolution launch (kind, M, N, "
        "K, minimum HBM bytes) to this file, for scripts/gemm_roofline.py", "ops"),
    Var("CLOUD_AMD_BN_FOLD", bool, True, "ResNet block backward: the bn3 / bn1 backward apply runs in the operand "
        "fetch of the 1x1 input-gradient GEMM that consumes it (ca_gemm_xa.h) instead of a separate pass", "ops"),
    Var("CLOUD_AMD_BN_FOLD_FWD", bool, True, "ResNet block forward: bn2's apply runs in conv3's operand fetch and "
        "bn3's (+ residual) in the next block's conv1 (ca_gemm_xa.h); the applied tensors are written once, by "
        "those GEMMs", "ops"),
    Var("CLOUD_AMD_BN_FOLD_MAX_N", int, 256, "BN fold sites kept: only GEMMs with K >= 2N and N <= this "
        "(ResNet-50 default: bn3 -> conv3 dgrad and bn3 -> next conv1 at stages 1-3, the stage-3 ones on the two-deep "
        "128 x 256 transform-A tiles, CLOUD_AMD_XA_N256=3: +0.6 / +1.0 % on two boxes, docs/performance.md round 6; "
        "4096 = every stage); the short-K sites (bn2 -> conv3, bn1 -> conv1 dgrad) measured slower than the separate "
        "pass, and stage 4 (N 512) +0.3 % below stages 1-3 only", "ops"),
    Var("CLOUD_AMD_BN_FOLD_WGRAD", bool, True, "bn3 -> conv3 fold at 64 input channels (ResNet stage 1): conv3's weight "
        "gradient runs in the same kernel as its input gradient (ca_gemm_xa.h mfma_gemm_xa_dw), so the BN-backward "
        "output dz3 is never written", "ops"),
    Var("CLOUD_AMD_BN_FOLD_DS", bool, False, "ResNet projection blocks, stages 2-4: the shortcut BN's backward apply "
        "runs in the operand fetch of the sparse strided shortcut input-gradient GEMM (ca_gemm_xa_bwd_strided); A/B",
        "ops"),
    Var("CLOUD_AMD_DS_SPARSE_DGRAD", bool, True, "ResNet projection blocks with a strided 1x1 shortcut: the "
        "shortcut's input gradient is written for its one non-empty output-parity class only, and conv1's input "
        "gradient accumulates into it reading the other pixels as zeros -- no zero-fill of 3/4 of dx and no read "
        "of those zeros", "ops"),
    Var("CLOUD_AMD_BN_FOLD_WGRAD_DS", bool, True, "stage-1 projection shortcut: its BN backward (gated by the block "
        "output's ReLU mask), the shortcut conv's input gradient and its weight gradient in one pass", "ops"),
    Var("CLOUD_AMD_BN_FOLD_WGRAD2", bool, False, "the same one-pass input + weight gradient for stage 2's conv3 "
        "(K = 512 -> N = 128, 8-wave workgroups holding the 512 x 128 dW block)", "ops"),
    Var("CLOUD_AMD_BN_FOLD_WGRAD1", bool, False, "the same one-pass input + weight gradient for stage 1's conv1 with "
        "bn1's backward apply (K = 64 -> N = 256: dz1 never written, four output chunks per tile)", "ops"),
    Var("CLOUD_AMD_XA_N256", int, 3, "transform-A GEMMs (BN folded into a 1x1 conv) with N a multiple of 256: "
        "1 = 128 x 256 tiles on 16-wave workgroups (each A tile transformed once), 2 = 128 x 256 on 8 waves "
        "(CLOUD_AMD_BUILD_EXPERIMENTAL builds only), "
        "3 = 16 waves with two K tiles' operands in flight (coefficients staged in LDS; K <= 2048), "
        "0 = 128 x 128 tiles.  Only the fold sites CLOUD_AMD_BN_FOLD_MAX_N admits reach them (ResNet-50 stage 3 "
        "at the default; measured in docs/performance.md, round 6)", "ops"),
    Var("CLOUD_AMD_XA_WAVES", int, 8,"128 x 128 transform-A GEMMs (BN folded into the 1x1 convs): 8-wave "
        "workgroups (<= 128 registers, two per CU) or 4", "ops"),
    Var("CLOUD_AMD_XA_WAVES_N64", bool, True, "the 128 x 64 transform-A GEMMs (stage 1) on 8-wave workgroups too "
        "(with CLOUD_AMD_XA_WAVES=8)", "ops"),
    Var("CLOUD_AMD_XA_DW_WAVES", int, 4, "stage-1 conv3 fused input+weight gradient: 4-wave workgroups (two per "
        "CU) or 8 (one per CU); 8 selects the one-step form", "ops"),
    Var("CLOUD_AMD_XA_DW_DEPTH", int, 1, "stage-1 fused input+weight gradient (K 256 -> N 64): 0 = one-step form; "
        "1, 2, 4 = deep form (weights resident in LDS, epilogue operands ahead of the next tile's) with that many "
        "source steps in flight per workgroup (1: two workgroups per CU, 2 and 4: one)", "ops"),
    Var("CLOUD_AMD_BN_FOLD_ALL", bool, False, "fold every BN site regardless of CLOUD_AMD_BN_FOLD_MAX_N (tests, A/B)",
        "ops"),
    Var("CLOUD_AMD_MAX_STEPS_IN_FLIGHT", int, 2, "training loops (benches, Keras fit) let the host enqueue at most this "
        "many steps ahead of the GPU (runtime.step_pacer); bounds the memory in flight so the caching allocator "
        "stops requesting segments after warmup; 0 = unbounded", "runtime"),
    Var("CLOUD_AMD_RUN_AHEAD_MS", float, 25.0, "the step pacer deepens its bound (up to 4 steps) so the queued steps "
        "cover at least this much GPU time, measured on the first steps: short steps (BERT-base 8.7 ms -> 3) "
        "absorb host hiccups, long ones keep CLOUD_AMD_MAX_STEPS_IN_FLIGHT; 0 = fixed depth", "runtime"),
    Var("CLOUD_AMD_GC_FREEZE", bool, True, "training loops (benches, Keras fit) call runtime.gc_control.freeze() after "
        "their first steps: objects alive then are excluded from Python's full collections", "runtime"),
    Var("CLOUD_AMD_WGRAD_STREAM", bool, True, "ResNet block / BERT layer backward: weight-gradient GEMMs on a "
        "second HIP stream, overlapping the memory-bound BN/LN/dgrad chain", "ops"),
    Var("CLOUD_AMD_BN_BWD_EPILOGUE", bool, True, "ResNet block backward: BatchNorm-backward statistics from the "
        "dgrad GEMM epilogues (skips the BN reduction pass)", "ops"),
    Var("CLOUD_AMD_REPO", str, None, "example notebooks: repository root to put on sys.path", "examples"),
    Var("CLOUD_AMD_DEBUG_SYNC", bool, False, "debug: synchronise after every native kernel launch so a fault is "
        "reported by the op that caused it; run() also sets HIP_LAUNCH_BLOCKING/AMD_SERIALIZE_KERNEL", "ops"),
    Var("CLOUD_AMD_PRECISION", str, "auto", "Keras dtype policy: auto (mixed_bfloat16 on an MI355X, float32 on "
        "CPU) | float32 | mixed_bfloat16 | bfloat16", "ops"),
    Var("CLOUD_AMD_ARCH", str, "gfx950", "offload arch of the native build", "build"),
    Var("CLOUD_AMD_SANITIZE", bool, False, "build the C++ test binary with ASan/UBSan", "build"),
    # distributed
    Var("CLOUD_AMD_COMM", str, "torch", "DP transport: 'torch' (torch.distributed/RCCL) or 'rccl' (native)",
        "distributed"),
    Var("CLOUD_AMD_DIST_BACKEND", str, None, "process-group backend override ('gloo' / 'nccl'); default nccl "
        "(RCCL) on GPU, gloo on CPU", "distributed"),
    Var("CLOUD_AMD_SHARED_GPU", bool, False, "rehearsal: every local rank uses cuda:0 (pair with "
        "CLOUD_AMD_DIST_BACKEND=gloo on a one-GPU box)", "distributed"),
    Var("CLOUD_AMD_BUCKET_MB", float, 16.0, "gradient bucket size (MB) of the DP engine", "distributed"),
    Var("CLOUD_AMD_STEM_TAIL", bool, True, "ResNet stem: BN + ReLU + max-pool fused (fwd) and max-pool backward "
        "fused with the BN-backward statistics", "ops"),
    Var("CLOUD_AMD_GRAD_FIN_BATCH", bool, True, "BERT layer backward: the eight fixed-order gradient "
        "finalisations (split-K slab sums, LayerNorm / bias column partials) run as ONE launch at the end of the "
        "layer (csrc/kernels/gradfin.hip); 0 = one launch each", "ops"),
    Var("CLOUD_AMD_LN_BIAS_FWD", bool, True, "BERT: the LayerNorm forward adds the bias of the output projection "
        "that feeds it (attention output, FFN2), so those GEMMs run without a bias epilogue", "ops"),
    Var("CLOUD_AMD_LN_BIAS_SUM", bool, True, "BERT: the LayerNorm backward also sums the bias gradient of the "
        "projection that fed it (no separate column-sum pass)", "ops"),
    Var("CLOUD_AMD_TAIL_BUCKET_MB", float, 1.0, "cap on the last gradient bucket (the first layers' gradients, "
        "ready only when backward ends: its all-reduce is exposed)", "distributed"),
    Var("CLOUD_AMD_SLICED_OPT", bool, False, "multi-GPU: run the fused optimizer update per gradient bucket as "
        "each bucket's all-reduce completes (overlapping the next bucket's), instead of once after the last one "
        "(opt-in until a multi-GPU run has shown it bitwise equal to the whole step and faster: the bench's N > 1 "
        "A/B cells measure both)",
        "distributed"),
    Var("CLOUD_AMD_TAPE_REDUCE", str, "overlap", "custom loops under a multi-replica strategy: 'overlap' -- "
        "tf.GradientTape.gradient returns the cross-replica SUM, all-reduced bucket by bucket during backward "
        "(Horovod DistributedGradientTape semantics); 'replica' -- per-replica gradients, summed in "
        "apply_gradients (TF MirroredStrategy semantics: a clip between the two sees one replica's gradient)",
        "distributed"),
    Var("CLOUD_AMD_SPLIT_PARAM_MB", float, 0.0, "a parameter larger than this is all-reduced as >= "
        "CLOUD_AMD_SPLIT_PARAM_MIN sub-buckets of about one bucket each, pipelined with the per-bucket optimizer "
        "(0 / unset: twice the bucket size)", "distributed"),
    Var("CLOUD_AMD_SPLIT_PARAM_MIN", int, 4, "minimum chunks of a split parameter", "distributed"),
    Var("CLOUD_AMD_BENCH_AB", str, "1", "benches at N > 1: DP-engine A/B cells after the timed region ('0' off, "
        "'1' the 12 default cells, or 'transport:bucket_mb:sliced,...')", "bench"),
    Var("CLOUD_AMD_SLICED_OPT_WORLD1", bool, False, "one GPU: start each gradient bucket's optimizer slice as soon "
        "as its gradients are final, beside the rest of backward (measured slower on MI355X: off by default)",
        "distributed"),
    Var("CLOUD_AMD_GRAD_REDUCE_DTYPE", str, "auto", "wire dtype of the gradient all-reduce: 'bf16' (every "
        "bucket, fp32 arenas through a bf16 copy: half the bytes), 'fp32' (every bucket through fp32), 'native' "
        "(each arena in its own dtype), 'auto' (= native: fp32 master-weight gradients keep fp32 sums; 'bf16' is "
        "the opt-in)",
        "distributed"),
    Var("CLOUD_AMD_RCCL_ENV", bool, True, "launcher sets the xGMI RCCL defaults (NCCL_MIN_NCHANNELS, "
        "HSA_NO_SCRATCH_RECLAIM) for multi-GPU jobs", "distributed"),
    Var("CLOUD_AMD_RCCL_CHANNELS", int, 0, "NCCL_MIN_NCHANNELS the launcher sets (0 = one per xGMI link)",
        "distributed"),
    Var("CLOUD_AMD_KFD_ROOT", str, "/sys/class/kfd/kfd/topology/nodes", "KFD topology root read by the "
        "node probe (tests point it at a fake tree)", "launcher"),
    Var("CLOUD_AMD_TUNER_STANDBY", bool, True, "trial scheduler: start the packing wave's workers with the probe "
        "wave, gated (imports done, no GPU touched) until the measured footprint says how many may run", "tuner"),
    Var("CLOUD_AMD_TUNER_STANDBY_PER_GPU", int, 8, "trial scheduler: at most this many gated standbys per GPU "
        "(and never more than max_workers - GPUs)", "tuner"),
    Var("CLOUD_AMD_TUNER_GATE_TIMEOUT_S", float, 600.0, "a gated standby tuner worker exits after waiting this long "
        "for the scheduler's verdict (it also exits when the scheduler is gone)", "tuner"),
    Var("CLOUD_AMD_TUNER_STANDBY_HIP", bool, False, "gated standby tuner workers also create their HIP context and "
        "load the kernel library before the gate opens (measured neutral on the 8-trial bench, "
        "profiles/r3_s28/: off by default, so a dismissed standby never touches the GPU)", "tuner"),
    Var("CLOUD_AMD_TUNER_FAST_EXIT", bool, True, "tuner workers end with os._exit after their last trial is in the "
        "study (no interpreter / HIP teardown on the study's critical path)", "tuner"),
    Var("CLOUD_AMD_TUNER_EARLY_FOOTPRINT", bool, True, "tuner probe worker: report the trial HBM footprint after "
        "the first training step of its first trial (0 = after the whole trial)", "tuner"),
    Var("CLOUD_AMD_TRIAL_DEVICE", str, None, "device of a tuner worker (set by TrialScheduler); recorded on every "
        "trial it runs in the study", "tuner"),
    Var("CLOUD_AMD_SCHED_FAKE_DEVICES", bool, False, "TrialScheduler placement rehearsal on a CPU host: workers keep "
        "their assigned cuda:<i> name for the study record but compute on CPU (tests)", "tuner"),
    Var("CLOUD_AMD_FOOTPRINT_FILE", str, None, "where a tuner worker reports its first trial's peak HBM "
        "(set by TrialScheduler for the probe wave)", "tuner"),
    Var("CLOUD_AMD_BENCH_VIA_RUN", bool, True, "bench scripts launch their ranks through cloud_amd.run()",
        "bench"),
    Var("CLOUD_AMD_SMALLK_BATCH", int, 1024, "bench/smallk_gemm.py: ResNet batch the GEMM shapes are taken at",
        "bench"),
    Var("CLOUD_AMD_BENCH_ALLOW_CPU", bool, False, "let bench.py run ResNet-50 on CPU (debug only)", "bench"),
    Var("CLOUD_AMD_DDP_ORDER", str, "event", "bucket ordering: 'event' (comm stream waits on a compute event), "
        "'sync' (debug), 'backend'", "distributed"),
    Var("CLOUD_AMD_GRAD_CHECK_EVERY", int, 0, "cross-rank gradient fingerprint check every N steps (0 = off)",
        "distributed"),
    # observability
    Var("CLOUD_AMD_TRACE", bool, False, "emit roctx ranges (forward/backward/allreduce/optimizer)", "observability"),
    Var("CLOUD_AMD_MONITORING_EXPORTER_ENABLED", bool, False, "start the C++ metrics exporter", "observability"),
    Var("CLOUD_AMD_MONITORING_PROJECT_ID", str, "", "project id stamped on exported series", "observability"),
    Var("CLOUD_AMD_MONITORING_METRICS_WHITELIST", str, "", "comma-separated metric allow-list", "observability"),
    Var("CLOUD_AMD_MONITORING_INTERVAL_S", float, 10.0, "export interval", "observability"),
    Var("CLOUD_AMD_MONITORING_SINK", str, "jsonl", "auto-started exporter sink: jsonl | prometheus",
        "observability"),
    Var("CLOUD_AMD_MONITORING_DIR", str, None, "exporter output directory (default: the job dir)", "observability"),
    # fault injection / tuner / data
    Var("CLOUD_AMD_FAULT", str, "", "fault injection 'rank:step:kind' (exit|raise|hang)", "testing"),
    Var("CLOUD_AMD_FAULT_HANG_S", float, 3600.0, "how long an injected hang sleeps", "testing"),
    Var("CLOUD_AMD_TUNER_ID", str, None, "tuner id of a scheduler worker", "tuner"),
    Var("CLOUD_AMD_TUNER_DIR", str, None, "default KerasTuner results directory", "tuner"),
    Var("CLOUD_AMD_STUDY_DIR", str, None, "local study-service directory", "tuner"),
    Var("CLOUD_AMD_HBM_GB", float, 288.0, "HBM per GPU used for trial packing", "tuner"),
    Var("CLOUD_AMD_DATA", str, None, "directory of real .npz datasets (else synthetic)", "data"),
    # benchmarks / examples
    Var("CLOUD_AMD_BENCH_BATCH", int, 1024, "per-GPU batch of bench.py (41 GB of the 288 GB HBM)", "bench"),
    Var("CLOUD_AMD_BUCKET_ORDER", str, "ready", "gradient buckets launch in backward-completion order across "
        "arenas ('ready', default) or in arena order ('arena')", "distributed"),
    Var("CLOUD_AMD_COMM_INIT_TIMEOUT_S", float, 300.0, "deadline for the native communicator's bootstrap (unique-id "
        "exchange + non-blocking init); past it the communicator is aborted and TimeoutError raised", "distributed"),
    Var("CLOUD_AMD_EXAMPLE_CPU", bool, False, "examples: launch CPU ranks instead of GPUs", "examples"),
    Var("CLOUD_AMD_EXAMPLE_SMALL", bool, False, "examples: tiny datasets (tests)", "examples"),
    Var("CLOUD_AMD_EXAMPLE_OUT", str, None, "examples: output directory", "examples"),
]

VARS = {v.name: v for v in _VARS}


def _parse(v: Var, raw: str):
    if v.type is bool:
        return raw.strip().lower() in ("1", "true", "yes", "on")
    return v.type(raw)


def get(name: str):
    """Typed value of a declared variable (its default when unset)."""
    v = VARS[name]
    raw = os.environ.get(name)
    if raw is None or raw == "":
        return v.default
    return _parse(v, raw)


def describe() -> str:
    rows = ["%-42s %-7s %-10s %s" % ("variable", "type", "default", "meaning")]
    for v in _VARS:
        rows.append("%-42s %-7s %-10s %s" % (v.name, v.type.__name__, v.default, v.doc))
    return "\n".join(rows)


if __name__ == "__main__":
    print(describe())
