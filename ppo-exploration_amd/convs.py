"""NatureCNN conv trunk on the libppox MFMA implicit-GEMM kernels.

Forward: ppox_nature_conv_fwd[_split] (fused u8->f32, bias, ReLU) for the three
convolutions of .ipynb_checkpoints/models-checkpoint.py:52-58, with activations
laid out NHWC between layers and NCHW at the trunk output (the reference's
Flatten order for Linear(3136, 512)).
Backward: libppox MFMA dgrad (ReLU backward of the layer below fused) and
split-K wgrad (+ bias grad, deterministic fixed-order reduction) kernels.

Math modes (PPOX_CONV_MATH, default "split"):
  "split" — f32 operands scaled per tensor by a power of two and split into two fp16
            planes on the f16 matrix cores, three products per multiply (csrc/conv.hip,
            csrc/conv_split.hip): fp32-class accuracy (at or below the f32-MFMA kernels'
            error vs fp64, tests/test_kernels_gpu.py).  The per-tensor scales come from
            "amax slots" that each producing kernel records into (one zeroed table per
            forward pass, AM_* rows below).  Ops without a split kernel yet use "f32".
  "split_all" — every op that has a split kernel, including those measured slower
            than their f32 kernel at the training batch (SPLIT_SLOWER; tests).
  "f32"   — v_mfma_f32_32x32x2_f32: every product an exact f32 FMA (csrc/conv.hip).
"""
import os

import torch

import native

MATHS = ("split", "split_all", "f32")
# ops that have a split-f16 kernel: ("fwd" | "dgrad" | "wgrad", layer)
SPLIT_OPS = {("fwd", 1), ("fwd", 2), ("fwd", 3), ("dgrad", 2), ("dgrad", 3), ("wgrad", 1), ("wgrad", 2), ("wgrad", 3)}
# ops whose split kernel exists but is not faster than the f32 one at the training batch
# (measured, tools/conv_bench.py); "split" mode runs them in f32.  conv2 dgrad left this set
# with its col2im-form kernel (dgrad2_col_kernel: 0.68 vs 0.97 ms f32 at B = 16384, 0.091 vs
# 0.136 ms at the 8-GPU per-rank minibatch of 2048)
SPLIT_SLOWER = set()
# fc forward: the split-f16 GEMM from FC_SPLIT_MIN_BATCH up (rocBLAS below; PPOX_FC_SPLIT_MIN
# overrides, default: every batch), split over K below FC_SPLITK_MAX_BATCH (tools/fc_bench.py,
# r02: split-K 0.018 / 0.045 / 0.078 ms vs rocBLAS 0.026 / 0.062 / 0.119 ms at 512 / 2048 /
# 4096 rows; the plain split GEMM 0.146 vs split-K 0.152 ms at 8192)
FC_SPLIT_MIN_BATCH = int(native.ab_env("PPOX_FC_SPLIT_MIN", "0"))
FC_SPLITK_MAX_BATCH = int(native.ab_env("PPOX_FC_SPLITK_MAX", "8192"))
# fc dgrad fused with the trunk's ReLU backward + NHWC transpose (split-f16) up to this
# batch (PPOX_FC_DGRAD_FUSED_MAX overrides): faster than rocBLAS + nchw_to_nhwc_mask at
# every measured batch (A/B: -33 ms per iteration at 16384, -2 ms at 2048)
FC_DGRAD_FUSED_MAX_BATCH = int(native.ab_env("PPOX_FC_DGRAD_FUSED_MAX", str(1 << 62)))
# fc weight gradient on the split wgrad kernel (ppox_nature_fc_wgrad) from this batch up,
# the rocBLAS f32 GEMM + NHWC -> Flatten permute below (PPOX_FC_WGRAD_SPLIT_MIN overrides)
FC_WGRAD_SPLIT_MIN_BATCH = int(native.ab_env("PPOX_FC_WGRAD_SPLIT_MIN", "0"))

# the heads' hidden layer Linear(512, 512) on the split-f16 GEMM (ppox_head_hidden_*) from this
# batch up, rocBLAS f32 below (PPOX_HEAD_SPLIT_MIN overrides)
HEAD_SPLIT_MIN_BATCH = int(native.ab_env("PPOX_HEAD_SPLIT_MIN", "8192"))
# below HEAD_SPLIT_MIN_BATCH the hidden layer's forward still runs on the split-f16 kernel, split over K
# with the critic head fused into its reduce (its backward stays on the library GEMMs);
# PPOX_HEAD_FWD_SPLITK=0 keeps the library GEMM
HEAD_FWD_SPLITK = native.ab_env("PPOX_HEAD_FWD_SPLITK", "1") == "1"
# the hidden layer's backward (dgrad into the fc layer's input grad + weight gradient) on the split-f16
# kernels from this batch up, the library GEMMs below (PPOX_HEAD_BWD_SPLIT_MIN).  Round 4: at every batch —
# the same GPU time at the per-rank 2,048 rows (same-box A/B 199.57 vs 199.55-199.79 ms per iteration,
# profiles/r04_ab.txt) and no library GEMM on the host's launch path (the two rocBLAS calls cost ~100 us of
# host time per minibatch, which the 8-rank path spends on its collectives)
HEAD_BWD_SPLIT_MIN_BATCH = int(native.ab_env("PPOX_HEAD_BWD_SPLIT_MIN", "0"))

# ReLU masks of the conv outputs as bitmasks written by the split forwards for the split dgrads
# (PPOX_RELU_BITS=0: the dgrads read the f32 activations)
RELU_BITS = native.ab_env("PPOX_RELU_BITS", "1") != "0"

# rows of a pass's amax table (native.amax_table): the split-f16 operands of the trunk and the
# heads' hidden layer, each recorded by the kernel that produces it and read by its consumers;
# row AM_EXP holds the exponents of the pass's PX tensors (slots EX_*)
AM_H1, AM_H2, AM_H3, AM_DF, AM_G3, AM_G2, AM_G1, AM_F, AM_DE, AM_EXP = range(10)
AM_ROWS = 10
EX_H2, EX_H3, EX_G3, EX_DF, EX_G2 = range(5)

# PX (round 4, include/ppox.h): in split math the trunk's other split operands are stored as their
# two f16 planes too — h2 (written by the conv2 forward, read by the conv3 forward and weight
# gradient), h3 (conv3 forward -> fc forward and fc weight gradient) and g3 (fc dgrad -> conv3
# dgrad and weight gradient) — at exponents derived from bounds, so no consumer splits in
# registers.  PPOX_PX=0: f32 tensors (split in the consumers).  Needs the ReLU bitmasks (the
# dgrads' masks cannot come from planes).
PX = native.ab_env("PPOX_PX", "1") != "0"
# ... from this batch up (PPOX_PX_MIN): every batch since the direct conv2 / conv3 forwards (csrc/dconv.hip,
# which need the planes; same-box A/B: 1-GPU line 478.6k vs 469.9k env-steps/s — the collect forward at 4,096
# rows gains most — and per-rank 204.8 vs 207.3 ms; before them PX at 2,048 rows measured 225.8 vs 219.5 ms)
PX_MIN_BATCH = int(native.ab_env("PPOX_PX_MIN", "0"))
# PX df (round 4, PPOX_PX_DF=1): the fc layer's df (B x 512, its amax recorded by the head backward)
# split into its planes by one small kernel (ppox_px_split) for the fc dgrad and weight gradient, which
# otherwise split every df value in registers once per tile (the fc dgrad: 49 times).  On by default
# since the direct fc dgrad (csrc/dconv.hip fcd_kernel, which reads the planes: 195 vs 277 us at 16,384
# rows); with the sg2 fc dgrad alone it measured neutral-to-slower (profiles/r04_ab.txt: 1-GPU 1,152.5
# vs 1,146.8 ms, per-rank 203.9 vs 201.8 ms per iteration)
PX_DF = native.ab_env("PPOX_PX_DF", "1") == "1"
# PX g2 + the direct conv2 dgrad (round 5, PPOX_DDGRAD2=1 by default): the conv3 dgrad writes g2 as its
# planes (bound: amax(g3) x the conv3 dgrad matrix's column norms), read as they lie by the direct
# class-wise conv2 dgrad (csrc/dconv.hip ddgrad2_kernel: per input-pixel parity class an implicit GEMM
# over its 4 taps x 64 channels, no col2im) and by the conv2 weight gradient; =0: f32 g2, the persistent
# col2im dgrad (dgrad2_colp_kernel)
DDGRAD2 = native.ab_env("PPOX_DDGRAD2", "1") != "0"


class PassState:
    """Side data of one trunk pass for the split kernels: the amax table (pass[AM_*] is its row),
    the ReLU bitmasks of the three conv outputs (bits[l - 1] for layer l: int32 words per
    output pixel, bit c % 32 of word c / 32 = channel c > 0; None unless that split forward wrote
    it), which the next layer's dgrad reads instead of the f32 activations, and which of h2, h3,
    g3 the pass holds as PX planes (px[EX_*]; their exponents: exp(EX_*))."""

    __slots__ = ("amax", "bits", "px")

    def __init__(self, amax, bits=(None, None, None), px=(False, False, False, False, False)):
        self.amax, self.bits, self.px = amax, bits, list(px)

    def __getitem__(self, row):
        return self.amax[row]

    def exp(self, which):
        """the int32 element holding PX tensor `which`'s exponent, or None when it is f32"""
        return self.amax[AM_EXP, which:which + 1] if self.px[which] else None


# backward on two streams: each layer's weight gradient runs on a side stream beside the
# main stream's dgrad chain (wgrad3 || dgrad3, wgrad2 || dgrad2; the fc weight gradient ||
# the fc dgrad), joined before the optimizer reads the gradients (PPOX_BWD_STREAMS=0: one stream)
BWD_STREAMS = native.ab_env("PPOX_BWD_STREAMS", "1") != "0"
BWD_SOLO_DGRAD2_BATCH = int(native.ab_env("PPOX_BWD_SOLO_DGRAD2", str(1 << 62)))
# PPOX_FORK_LATE=1: below that batch the conv2 weight gradient's side-stream wait (on the point after the
# conv3 dgrad) is enqueued after the conv2 dgrad's launch instead of before it — the same dependencies,
# another capture order for a hipGraph of the pass (tools/graph_probe.py)
FORK_LATE = native.ab_env("PPOX_FORK_LATE", "0") == "1"
# PPOX_FORK_MERGE=1: the heads' hidden-layer weight gradient joins the fc weight gradient's fork to the side
# stream (one main-stream event record per minibatch fewer; models.CnnActorCritic.backward_train)
FORK_MERGE = native.ab_env("PPOX_FORK_MERGE", "0") == "1"
# PPOX_BWD_SOLO_WGRAD2=1: from that batch conv2's weight gradient also runs alone on the main stream
# (after the dgrad, before wgrad1) instead of beside wgrad1 — 1 % slower (same-box A/B), but its
# event time is then its own execution time
BWD_SOLO_WGRAD2 = native.ab_env("PPOX_BWD_SOLO_WGRAD2", "0") != "0"
SIDE_PRIO = native.ab_env("PPOX_SIDE_PRIO", "0" if native.ab_env("PPOX_TRAIN_PRIO", "0") == "1" else "1") == "1"
_side = {}


def side_stream(device, k=0):
    """Side stream k of `device` (0: the concurrent weight-gradient kernels; 1: PPO_ICM's
    curiosity-module work beside the policy minibatch)."""
    s = _side.get((device, k))
    if s is None:
        # high priority: HIP multiplexes the streams of one priority class over GPU_MAX_HW_QUEUES hardware
        # queues, and two streams on one queue run in order — in the main stream's class (the default
        # stream) a pooled stream may land on the main stream's queue, as it did once RCCL had created
        # its streams (per-rank 196 -> 242 ms); PPOX_SIDE_PRIO=0: default priority
        s = torch.cuda.Stream(device=device, priority=-1 if SIDE_PRIO else 0)
        _side[(device, k)] = s
    return s


_events = {}
_cur_streams = {}


def current_stream(device):
    """torch.cuda.current_stream(device) without its per-call device-index and Stream-object cost
    (~10 us: the backward forks / joins the side stream several times per minibatch): torch's own
    Stream object of the current raw stream, looked up once per (device, raw stream).  (Not an
    ExternalStream: wrapping the default stream's handle 0 makes a new stream, which breaks the
    fork / join ordering — tests/test_kernels_gpu.py::test_current_stream_orders_like_torch.)"""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    raw = torch._C._cuda_getCurrentRawStream(idx)
    s = _cur_streams.get((idx, raw))
    if s is None:
        s = _cur_streams[(idx, raw)] = torch.cuda.current_stream(idx)
    return s


def _event(side, which):
    # one reusable event per (side stream, direction): a wait takes the event's most recent
    # record at the time it is enqueued, so re-recording it for the next fork / join is safe
    ev = _events.get((side, which))
    if ev is None:
        ev = _events[(side, which)] = torch.cuda.Event()
    return ev


# PPOX_EVENT_FENCE: the fork / join events' fence — "system" (default: native events with HIP's default, a
# system-scope release on every record), "device" (hipEventReleaseToDevice), "none" (hipEventDisableSystemFence),
# "torch" (torch's events).  "none" ran the per-rank shape ~1 % faster (profiles/r05g: 190.9 -> 188.8 ms) and
# was the default in round 5, but a kernel on one stream then reads another stream's fresh output stale now and
# then: the 8-rank C4 run (tests/test_c4_gpu.py, every update teacher-forced) found non-finite df planes and
# conv gradients in about one rank pass in 200 under it, none under "system" or one stream (round 6)
EVENT_FENCE = native.ab_env("PPOX_EVENT_FENCE", "system")
_nevents = {}


def _order(side, which, rec, wait):
    ev = _nevents.get((side, which))
    if ev is None:
        flags = {"device": native.EVENT_RELEASE_TO_DEVICE, "none": native.EVENT_DISABLE_SYSTEM_FENCE}.get(EVENT_FENCE, 0)
        ev = _nevents[(side, which)] = native.event_create(flags)
    native.stream_order(ev, rec, wait)


def fork(side, cur=None):
    """side waits for everything enqueued so far on `cur` (default: the current stream)."""
    if EVENT_FENCE != "torch":
        _order(side, 0, cur if cur is not None else torch.cuda.current_stream(), side)
        return
    ev = _event(side, 0)
    ev.record(cur)
    side.wait_event(ev)


def join(side, cur=None):
    """`cur` (default: the current stream) waits for everything enqueued so far on side."""
    if EVENT_FENCE != "torch":
        _order(side, 1, side, cur if cur is not None else torch.cuda.current_stream())
        return
    ev = _event(side, 1)
    ev.record(side)
    (cur if cur is not None else torch.cuda.current_stream()).wait_event(ev)


def default_math():
    m = os.environ.get("PPOX_CONV_MATH", "split")
    if m not in MATHS:
        raise ValueError(f"PPOX_CONV_MATH must be one of {MATHS}, got {m!r}")
    return m


class RolloutRows:
    """Minibatch observations left in the rollout: rows idx (env-major i = env * T + step,
    device int64) of the step-major (T, N, 4, 84, 84) uint8 frame buffer.  The split conv1
    kernels read them in place (ppox_nature_conv_fwd_split / _wgrad_split_idx with idx), so
    the minibatch gather (ppox_gather_rows, 2 x 28,224 B per row) is not run."""

    dtype = torch.uint8

    def __init__(self, frames, idx):
        assert frames.dtype == torch.uint8 and frames.dim() == 5 and frames.is_contiguous()
        self.frames, self.idx = frames, idx.contiguous()
        self.T, self.N = int(frames.shape[0]), int(frames.shape[1])
        self.shape = (int(idx.numel()),) + tuple(frames.shape[2:])
        self.device = frames.device

    def contiguous(self):
        return self


class _NatureTrunk(torch.autograd.Function):
    """Autograd wrapper of the trunk (tests, non-explicit nets): returns h3 in the reference's
    (B, 64, 7, 7) layout — a permuted view of the NHWC h3 in split math."""

    @staticmethod
    def forward(ctx, x, convs, w1, b1, w2, b2, w3, b3):
        h1, h2, h3, am = convs.forward_acts(x, train=True, px=False)  # (h3 is returned to autograd as f32)
        ctx.convs, ctx.am = convs, am
        ctx.save_for_backward(x, h1, h2, h3)
        return h3.permute(0, 3, 1, 2) if convs.nhwc3 else h3

    @staticmethod
    def backward(ctx, dh3):
        x, h1, h2, h3 = ctx.saved_tensors
        am = ctx.am
        convs = ctx.convs
        grads = [torch.zeros_like(t) for t in (convs.c1.weight, convs.c1.bias, convs.c2.weight, convs.c2.bias,
                                               convs.c3.weight, convs.c3.bias)]
        if convs.nhwc3:
            g3 = dh3.permute(0, 2, 3, 1).contiguous()
            native.relu_backward_(g3, h3, amax=am[AM_G3])
            convs.backward_acts(x, h1, h2, h3, None, *grads, g3=g3, am=am)
        else:
            convs.backward_acts(x, h1, h2, h3, dh3.contiguous(), *grads, am=am)
        return (None, None, *grads)


class WmaxLink:
    """The weight packing's amax pass folded into the Adam step (round 6): the packing of
    the five NatureCNN weight tensors needs each tensor's max |w| before it can split a value, which took a
    launch of its own (wmax_kernel) at every optimizer step.  FlatParams.adam_step records the maxima of the
    weights it writes (ppox_adam_step_wmax) into bufs[nxt], which the packing zeroed beforehand; the next
    packing of those same weights (same step count, buffer and torch version counter) reads them and runs as one
    launch (ppox_nature_pack_all_wmax), zeroing the other buffer for the next step.  Anything else packs with its
    own amax pass: weights written in place after the step (a torch in-place op on the flat buffer or a view of
    it bumps the buffer's version counter, one through a weight Parameter — load_state_dict — the Parameter's;
    both are part of the key), invalidate(), two steps without a packing between."""

    def __init__(self, flat, weights):
        base, n = flat.data.data_ptr(), flat.data.numel()
        offs = [(w.data_ptr() - base) // 4 for w in weights]
        for w, o in zip(weights, offs):
            if not (w.is_contiguous() and w.dtype == torch.float32 and 0 <= o and o + w.numel() <= n):
                raise ValueError("WmaxLink: the weights must be contiguous f32 views of the flat buffer")
        self.ranges = torch.tensor(offs + [w.numel() for w in weights], dtype=torch.int64)
        self.weights = tuple(weights)
        self.folds = 0  # packings that read the step's partials (tests)
        self.bufs = torch.zeros(2, native.WMAX_TENSORS * native.WMAX_SLOTS, dtype=torch.int32, device=flat.device)
        self.zeroed = [True, True]
        self.nxt = 0
        self.valid = None  # (step count, data pointer, torch version, buffer) of the last recorded maxima

    def ready(self, flat):
        """the buffer the next step records into is zeroed"""
        return self.zeroed[self.nxt]

    def recording(self):
        return self.bufs[self.nxt]

    def _key(self, flat):
        return (flat.step_count, flat.data.data_ptr(), flat.data._version) + tuple(w._version for w in self.weights)

    def recorded(self, flat):
        self.valid = (self._key(flat), self.nxt)
        self.zeroed[self.nxt] = False

    def for_pack(self, flat):
        """(amax_in or None, amax_next) for a packing of the weights as they are now"""
        if self.valid is not None and self.valid[0] == self._key(flat):
            i = self.valid[1]
            self.nxt = i ^ 1
            amax_in = self.bufs[i]
            self.folds += 1
        else:
            self.valid = None
            amax_in = None
        self.zeroed[self.nxt] = True  # zeroed by the packing launch (stream order: before the next step)
        return amax_in, self.bufs[self.nxt]

    def invalidate(self):
        self.valid = None


class NatureConvs:
    """Callable conv trunk bound to a CnnActorCritic whose parameters live in a FlatParams."""

    def __init__(self, net, flat, math=None):
        fe = net.feature_extractor
        self.c1, self.c2, self.c3 = fe[0], fe[2], fe[4]
        self.flat = flat
        self.math = math or default_math()
        if self.math not in MATHS:
            raise ValueError(f"math must be one of {MATHS}")
        dev = flat.device
        self.wp1 = torch.empty(256 * 32, device=dev)
        self.wp2 = torch.empty(512 * 64, device=dev)
        self.wp3 = torch.empty(576 * 64, device=dev)
        self.wpd2 = torch.empty(4 * 256 * 32, device=dev)
        self.wpd3 = torch.empty(576 * 64, device=dev)
        # split-f16 planes (int16 storage), packed by ppox_nature_pack_split
        self.q = {k: torch.empty(native.nature_split_pack_elems(k), dtype=torch.int16, device=dev)
                  for k in (1, 2, 3, 12, 13)}
        # fc layer (feature_extractor[7], 3136 -> 512) split-f16 operands (split math only)
        self.fc = net.feature_extractor[7]
        nfc = native.nature_fc_pack_elems()
        self.qfc = (torch.empty(nfc, dtype=torch.int16, device=dev), torch.empty(nfc, dtype=torch.int16, device=dev)) \
            if self.math != "f32" else None
        # the heads' hidden layer (extra_layer[0], 512 -> 512): split-f16 forward / dgrad forms
        self.hid = net.extra_layer[0]
        nh = native.head_hidden_pack_elems()
        self.qh = (torch.empty(nh, dtype=torch.int16, device=dev), torch.empty(nh, dtype=torch.int16, device=dev)) \
            if self.math != "f32" else None
        # split math keeps conv3's output NHWC (B, 7, 7, 64): fc feature f = p * 64 + c is the
        # reference's Flatten feature c * 49 + p.  The split fc kernels are packed through that
        # permutation; the library GEMMs (fc forward below FC_SPLIT_MIN_BATCH, fc weight grad)
        # use this permuted f32 copy of the weight / permute their result back.
        self.nhwc3 = self.math != "f32"
        if self.nhwc3:
            f = torch.arange(3136, device=dev)
            self.fc_perm = (f % 64) * 49 + f // 64  # NHWC feature -> Flatten feature
            self.wfc_nhwc = torch.empty(512, 3136, device=dev)
        # split math: conv1's output h1 in the H1P form (its two f16 planes per value, 128 B per
        # pixel: csrc/conv_common.h) — written split by the conv1 forward at a scale derived from the
        # weights, read as it lies by the conv2 forward and the direct conv2 weight gradient
        self.h1p = self.math != "f32"
        # PX planes for h2 / h3 / g3 (see PX above) where the pass's ops all run split
        self.px = self.h1p and PX and RELU_BITS
        self._ws = {}
        self._diag = None  # a dict: the backward keeps its intermediates there (tests)
        self._version = None
        self._packed = set()
        self._last_batch = None
        self._forms_cache = {}
        # the Adam step records the packing's amax partials (split math; PPOX_WMAX_FOLD=0 under PPOX_AB=1: the
        # packing's own amax pass at every step)
        self._wmax = None
        if self.math != "f32" and native.ab_env("PPOX_WMAX_FOLD", "1") != "0":
            self._wmax = WmaxLink(flat, (self.c1.weight, self.c2.weight, self.c3.weight, self.fc.weight,
                                         self.hid.weight))
        flat.wmax = self._wmax  # the flat's latest trunk (a re-attach replaces the link)

    def split_head(self, batch):
        """the heads' hidden layer on the split-f16 kernels for a `batch`-row pass"""
        return self.qh is not None and batch >= HEAD_SPLIT_MIN_BATCH

    def split_head_fwd(self, batch):
        """only the hidden layer's forward on the split-f16 kernel (split over K) for a `batch`-row pass"""
        return self.qh is not None and HEAD_FWD_SPLITK and 0 < batch < HEAD_SPLIT_MIN_BATCH

    def split_head_bwd(self, batch):
        """the hidden layer's backward (dgrad + weight gradient) on the split-f16 kernels"""
        return self.qh is not None and (batch >= HEAD_SPLIT_MIN_BATCH or batch >= HEAD_BWD_SPLIT_MIN_BATCH)

    def head_fwd_ws(self, batch):
        """the split-K hidden forward's workspace, one per batch size (a captured collect graph keeps
        its own)"""
        ws = self._ws.get(("head_sk", batch))
        if ws is None:
            ws = torch.empty(max(native.head_hidden_fwd_splitk_workspace_bytes(batch), 16), dtype=torch.uint8,
                             device=self.flat.device)
            self._ws[("head_sk", batch)] = ws
        return ws

    def uses_split(self, op, layer, batch=None):
        if self.math == "split_all":  # every op that has a split kernel (tests, benchmarks)
            return (op, layer) in SPLIT_OPS or (op, layer) in SPLIT_SLOWER
        if self.math != "split":
            return False
        return (op, layer) in SPLIT_OPS

    def h1p_exponent(self):
        """E of the current H1P packing (h1 * 2^E = hi + lo), read back from q1's tail (tests)."""
        tail = self.q[1][native.nature_split_pack_elems(1) - 2 * native.PACK_TAIL32:].view(torch.int32)
        return int(tail[native.AMAX_SLOTS + 1])

    def empty_h1(self, B, device):
        """conv1's output buffer of a B-row pass: H1P (int16 planes) in split math, f32 NHWC else."""
        if self.h1p:
            return torch.empty((B, 20, 20, 64), dtype=torch.int16, device=device)
        return torch.empty((B, 20, 20, 32), device=device)

    def px_h3(self, B, train):
        """h3 as PX planes in a B-row pass: its consumers (the fc forward, and in training the fc weight
        gradient and the fused fc dgrad reading h3's bitmask) all run the split kernels"""
        return self.px and B >= FC_SPLIT_MIN_BATCH and (
            not train or (B >= FC_WGRAD_SPLIT_MIN_BATCH and B < FC_DGRAD_FUSED_MAX_BATCH))

    def px_df(self, B):
        """df as PX planes (ppox_px_split) for the split fc dgrad and weight gradient"""
        return (PX_DF and self.px and self.nhwc3 and B >= FC_WGRAD_SPLIT_MIN_BATCH
                and B < FC_DGRAD_FUSED_MAX_BATCH)

    def px_g3(self, B, am):
        """g3 as PX planes: the fc dgrad is the fused split kernel with h3's bitmask, the conv3 dgrad runs
        split with conv2's bitmask"""
        return (self.px and B >= PX_MIN_BATCH and isinstance(am, PassState) and am.bits[2] is not None and am.bits[1] is not None
                and B < FC_DGRAD_FUSED_MAX_BATCH and self.uses_split("dgrad", 3, B) and self.uses_split("wgrad", 3))

    def px_g2(self, B, am):
        """g2 as PX planes: the conv3 dgrad (split, g3's amax and conv2's bitmask) writes them, the direct
        conv2 dgrad (conv1's bitmask) and the conv2 weight gradient (H1P) read them"""
        return (DDGRAD2 and self.px and isinstance(am, PassState) and am.bits[0] is not None
                and am.bits[1] is not None and self.uses_split("dgrad", 3, B) and self.uses_split("dgrad", 2, B)
                and self.h1p)

    def workspace(self, layer, batch, split=False):
        if split and layer == 2 and self.h1p:
            need = native.nature_conv2_wgrad_planes_workspace_bytes(batch)
        else:
            need = (native.nature_wgrad_split_workspace_bytes if split else native.nature_wgrad_workspace_bytes)(layer,
                                                                                                               batch)
        ws = self._ws.get(layer)
        if ws is None or ws.numel() < need:
            ws = torch.empty(need, dtype=torch.uint8, device=self.flat.device)
            self._ws[layer] = ws
        return ws

    def _forms(self, batch):
        """Weight layouts the kernels of a `batch`-row pass use: f32-packed ('wp1' .. 'wpd3'),
        split-packed ('q1' .. 'qd3') and the fc's split forms ('qfcf', 'qfcd')."""
        forms = set()
        for op, L in (("fwd", 1), ("fwd", 2), ("fwd", 3), ("dgrad", 2), ("dgrad", 3)):
            split = self.uses_split(op, L, batch)
            forms.add(("q" if split else "wp") + ("d" if op == "dgrad" else "") + str(L))
        if self.math != "f32":
            forms.add("qfcd")
            forms.add("qfcf" if batch >= FC_SPLIT_MIN_BATCH else "wfc_nhwc")
        if self.split_head(batch):
            forms |= {"qhf", "qhd"}
        elif self.split_head_fwd(batch):
            forms.add("qhf")
        if self.split_head_bwd(batch):
            forms.add("qhd")
        return forms

    def pack(self, batch=0, zero=None):
        """Pack the weights (once per optimizer step) into the layouts the kernels of a
        `batch`-row pass use; a later pass of another size packs only the forms still missing
        (one ppox_nature_pack_all call for the split and fc forms).  `zero` (int32 tensor) is
        zeroed by that call when it runs: returns True if it did."""
        v = (self.flat.step_count, self.flat.data.data_ptr())
        key = (batch, HEAD_SPLIT_MIN_BATCH, HEAD_FWD_SPLITK, HEAD_BWD_SPLIT_MIN_BATCH, FC_SPLIT_MIN_BATCH)  # (tests patch these)
        if v == self._version and key == self._last_batch:  # the hot path: several times per minibatch
            return False
        if v != self._version:
            self._version, self._packed = v, set()
        self._last_batch = key
        forms = self._forms_cache.get(key)
        if forms is None:
            forms = self._forms_cache[key] = frozenset(self._forms(batch))
        missing = forms - self._packed
        if not missing:
            return False
        zeroed = False
        w1, w2, w3 = self.c1.weight, self.c2.weight, self.c3.weight
        pick = lambda name, buf: buf if name in missing else None
        if missing & {"wp1", "wp2", "wp3", "wpd3"}:
            native.nature_pack_weights(w1, w2, w3, pick("wp1", self.wp1), pick("wp2", self.wp2), pick("wp3", self.wp3),
                                       None, pick("wpd3", self.wpd3))
        if missing & {"wpd2", "q1", "q2", "q3", "qd2", "qd3", "qfcf", "qfcd", "qhf", "qhd"}:
            q = self.q
            qfc = self.qfc or (None, None)
            qh = self.qh or (None, None)
            lk = self._wmax if self._wmax is not None and self.flat.wmax is self._wmax else None
            if lk is not None:
                amax_in, amax_next = lk.for_pack(self.flat)
                native.nature_pack_all_wmax(w1, w2, w3, self.fc.weight, pick("wpd2", self.wpd2), pick("q1", q[1]),
                                            pick("q2", q[2]), pick("q3", q[3]), pick("qd2", q[12]),
                                            pick("qd3", q[13]), pick("qfcf", qfc[0]), pick("qfcd", qfc[1]),
                                            self.hid.weight, pick("qhf", qh[0]), pick("qhd", qh[1]), b1=self.c1.bias,
                                            zero=zero, b2=self.c2.bias, b3=self.c3.bias, amax_in=amax_in,
                                            amax_next=amax_next)
            else:
                native.nature_pack_all(w1, w2, w3, self.fc.weight, pick("wpd2", self.wpd2), pick("q1", q[1]),
                                       pick("q2", q[2]), pick("q3", q[3]), pick("qd2", q[12]), pick("qd3", q[13]),
                                       pick("qfcf", qfc[0]), pick("qfcd", qfc[1]), self.hid.weight,
                                       pick("qhf", qh[0]), pick("qhd", qh[1]), b1=self.c1.bias, zero=zero,
                                       b2=self.c2.bias, b3=self.c3.bias)
            zeroed = zero is not None
        if "wfc_nhwc" in missing:
            torch.index_select(self.fc.weight.detach(), 1, self.fc_perm, out=self.wfc_nhwc)
        self._packed |= missing
        return zeroed

    def invalidate(self):
        self._version = None
        self._packed = set()
        self._last_batch = None
        if self._wmax is not None:
            self._wmax.invalidate()

    # -- per-op dispatch (layer 1 input: uint8 frames, sample stride 4*84*84 bytes).  am: the
    # pass's amax table; a split kernel reads its f32 operands' rows and records its output's, an
    # f32 kernel whose output feeds a split one has it recorded by ppox_amax
    def fwd(self, layer, x, B, bias, y, am):
        stride = 4 * 84 * 84 if layer == 1 else 0
        out_am = am[AM_H1 + layer - 1] if self.math != "f32" else None
        bits = am.bits[layer - 1] if isinstance(am, PassState) else None
        px = am.px if isinstance(am, PassState) else (False, False, False, False)
        # conv1 records h1's amax for the bound of a PX h2
        h1_am = out_am if layer == 1 and px[EX_H2] else None
        if isinstance(x, RolloutRows):
            assert layer == 1 and self.uses_split("fwd", 1)
            if self.h1p:
                native.nature_conv1_fwd_planes(x.frames, B, x.idx, x.T, x.N, 0, self.q[1], bias, y, relu_bits=bits,
                                               amax_y=h1_am)
            else:
                native.nature_conv_fwd_split(1, x.frames, B, x.idx, x.T, x.N, 0, self.q[1], bias, y, amax_y=out_am,
                                             relu_bits=bits)
            return
        if self.h1p and layer == 1:
            native.nature_conv1_fwd_planes(x, B, None, 0, 0, stride, self.q[1], bias, y, relu_bits=bits, amax_y=h1_am)
        elif self.h1p and layer == 2:
            native.nature_conv2_fwd_planes(x, self.q[1], B, self.q[2], bias, y, amax_y=out_am, relu_bits=bits,
                                           amax_x=am[AM_H1] if px[EX_H2] else None, y_exp=am.exp(EX_H2) if px[EX_H2] else None)
        elif self.uses_split("fwd", layer):
            native.nature_conv_fwd_split(layer, x, B, None, 0, 0, stride, self.q[layer], bias, y,
                                         amax_x=am[AM_H1 + layer - 2] if layer > 1 else None, amax_y=out_am,
                                         relu_bits=bits, x_exp=am.exp(EX_H2) if layer == 3 and px[EX_H2] else None,
                                         y_exp=am.exp(EX_H3) if layer == 3 and px[EX_H3] else None)
        else:
            wp = (self.wp1, self.wp2, self.wp3)[layer - 1]
            native.nature_conv_fwd(layer, x, B, None, 0, 0, stride, wp, bias, y)
            if out_am is not None:
                native.amax(y, out_am)

    def dgrad(self, layer, g, B, prev_act, out, am):
        self.pack(B)  # the conv2 dgrad form depends on the batch
        g_am, out_am = (am[AM_G3], am[AM_G2]) if layer == 3 else (am[AM_G2], am[AM_G1])
        if self.uses_split("dgrad", layer, B):
            bits = am.bits[layer - 2] if isinstance(am, PassState) else None
            if layer == 2 and self.h1p and bits is None:
                raise ValueError("conv2 dgrad on H1P needs conv1's ReLU bitmask (a training pass's PassState)")
            ps = isinstance(am, PassState)
            g_exp = am.exp(EX_G3 if layer == 3 else EX_G2) if ps else None
            y_exp = am.exp(EX_G2) if layer == 3 and ps else None
            native.nature_conv_dgrad_split(layer, g, B, self.q[10 + layer], prev_act, out, amax_g=g_am,
                                           amax_out=out_am, relu_bits=bits, g_exp=g_exp, y_exp=y_exp)
        else:
            if layer == 2 and self.h1p:
                raise ValueError("the f32 conv2 dgrad needs f32 activations; split math keeps h1 as H1P")
            native.nature_conv_dgrad(layer, g, B, self.wpd2 if layer == 2 else self.wpd3, prev_act, out)
            if self.math != "f32":
                native.amax(out, out_am)

    def wgrad(self, layer, x, B, g, dw, db, am, stream=None):
        stride = 4 * 84 * 84 if layer == 1 else 0
        g_am = am[(AM_G1, AM_G2, AM_G3)[layer - 1]]
        if isinstance(x, RolloutRows):
            assert layer == 1 and self.uses_split("wgrad", 1)
            native.nature_conv_wgrad_split_idx(1, x.frames, B, x.idx, x.T, x.N, g, self.workspace(1, B, True), dw, db,
                                               amax_g=g_am, stream=stream)
            return
        if layer == 2 and self.h1p:
            native.nature_conv2_wgrad_planes(x, self.q[1], B, g, self.workspace(2, B, True), dw, db, amax_g=g_am,
                                             g_exp=am.exp(EX_G2) if isinstance(am, PassState) else None,
                                             stream=stream)
        elif self.uses_split("wgrad", layer):
            px = layer == 3 and isinstance(am, PassState)
            native.nature_conv_wgrad_split(layer, x, B, stride, g, self.workspace(layer, B, True), dw, db,
                                           amax_x=am[AM_H1 + layer - 2] if layer > 1 else None, amax_g=g_am,
                                           x_exp=am.exp(EX_H2) if px else None, g_exp=am.exp(EX_G3) if px else None,
                                           stream=stream)
        else:
            native.nature_conv_wgrad(layer, x, B, None, 0, 0, stride, g, self.workspace(layer, B), dw, db, stream=stream)

    def forward_acts(self, x, train=False, px=None, table=None):
        """Trunk forward: (h1 NHWC, h2 NHWC, h3, am) — activations (ReLU applied) and the pass's
        PassState (the amax table's AM_* rows — the backward of the same pass records its
        gradients' rows — and, for a `train` pass, conv1's ReLU bitmask); h3 is
        NHWC (B, 7, 7, 64) in split math (self.nhwc3), NCHW (B, 64, 7, 7) in f32 math.  px (default
        self.px): h2 / h3 as PX planes (int16 (B, 9, 9, 128) / (B, 7, 7, 128)) where their consumers
        allow; am.px says which.  table: an already zeroed (AM_ROWS, AMAX_SLOTS) int32 amax table for the pass
        (the collect graph's per-step tables, zeroed by one fill per rollout)."""
        B = x.shape[0]
        dev = x.device
        px = (self.px if px is None else (px and self.px)) and B >= PX_MIN_BATCH
        # the pass's amax table: zeroed by the weight packing when this pass runs it (the first
        # pass after an optimizer step), by a fill otherwise
        if table is not None:
            self.pack(B)
        else:
            table = torch.empty((AM_ROWS, native.AMAX_SLOTS), dtype=torch.int32, device=dev)
            if not self.pack(B, zero=table):
                table.zero_()
        h1 = self.empty_h1(B, dev)
        px2, px3 = px, px and self.px_h3(B, train)
        h2 = torch.empty((B, 9, 9, 128), dtype=torch.int16, device=dev) if px2 else torch.empty((B, 9, 9, 64), device=dev)
        h3 = (torch.empty((B, 7, 7, 128), dtype=torch.int16, device=dev) if px3 else
              torch.empty((B, 7, 7, 64) if self.nhwc3 else (B, 64, 7, 7), device=dev))
        # the conv outputs' ReLU bitmasks where the forward and the consumer of the mask (the next
        # layer's dgrad; for conv3 the fc dgrad) both run split (training passes)
        consumer = (self.uses_split("dgrad", 2, B), self.uses_split("dgrad", 3, B),
                    self.nhwc3 and B < FC_DGRAD_FUSED_MAX_BATCH)
        # (conv1's is required on H1P, whose planes are no f32 mask)
        bits = tuple(torch.empty(B * P * C // 32, dtype=torch.int32, device=dev)
                     if train and (RELU_BITS or (L == 1 and self.h1p)) and self.uses_split("fwd", L) and
                     consumer[L - 1] else None
                     for L, P, C in ((1, 400, 32), (2, 81, 64), (3, 49, 64)))
        am = PassState(table, bits, (px2, px3, False, False, False))
        if B:
            self.fwd(1, x, B, self.c1.bias, h1, am)
            self.fwd(2, h1, B, self.c2.bias, h2, am)
            self.fwd(3, h2, B, self.c3.bias, h3, am)
        return h1, h2, h3, am

    # ---- fc layer (split math): forward and the dgrad fused with the trunk's ReLU backward
    def fc_forward(self, h3, am, actor=None):
        """f = relu(h3 @ W^T + b), h3 (B, 7, 7, 64) NHWC (split math): the split-f16 GEMM when
        the batch fills the chip (ceil(B/128) row tiles x 8 column blocks >= ~512 workgroups),
        split over K below, rocBLAS on the NHWC-permuted weight below FC_SPLIT_MIN_BATCH.
        actor = (w, b): returns (f, logits), logits = f w^T + b computed by the split-K form's
        reduce (<= 8 actions) or None (the caller runs the actor head)."""
        self.pack(h3.shape[0])
        B = h3.shape[0]
        logits = None
        h3_exp = am.exp(EX_H3) if isinstance(am, PassState) else None
        if B < FC_SPLIT_MIN_BATCH:
            assert h3_exp is None, "PX h3 feeds the split fc kernels only"
            f = torch._addmm_activation(self.fc.bias, h3.view(B, -1), self.wfc_nhwc.t())  # bias+ReLU fused
            if am is not None:  # f's amax for the heads' split hidden layer (ppox_head_hidden_fwd*)
                native.amax(f, am[AM_F])
            return f if actor is None else (f, logits)
        f = torch.empty((B, 512), device=h3.device)
        if B < FC_SPLITK_MAX_BATCH:
            # one workspace per batch size: the collect graph captures the collect batch's buffer
            # (allocated by the eager first collect), which a training batch must never replace
            ws = self._ws.get(("fc_sk", B))
            if ws is None:
                ws = torch.empty(max(native.nature_fc_fwd_splitk_workspace_bytes(B), 16), dtype=torch.uint8,
                                 device=h3.device)
                self._ws[("fc_sk", B)] = ws
            if actor is not None and actor[0].shape[0] <= 8 and actor[0].is_contiguous() and actor[0].data_ptr() % 16 == 0:
                logits = torch.empty((B, actor[0].shape[0]), device=h3.device)
            native.nature_fc_fwd_splitk(h3, B, self.qfc[0], self.fc.bias, ws, f, amax_h3=am[AM_H3], amax_f=am[AM_F],
                                        actor=actor if logits is not None else None, logits=logits, h3_exp=h3_exp)
        else:
            native.nature_fc_fwd(h3, B, self.qfc[0], self.fc.bias, f, amax_h3=am[AM_H3], amax_f=am[AM_F],
                                 h3_exp=h3_exp)
        return f if actor is None else (f, logits)

    def fc_dgrad_g3(self, df, h3, am, dfp=None):
        """g3 (B, 7, 7, 64) NHWC = (df @ W) * (h3 > 0), df = dL/df after the fc ReLU (its amax in
        am[AM_DF]; dfp: its PX planes, am.px[EX_DF]), h3 NHWC; records g3's amax."""
        B = df.shape[0]
        px = self.px_g3(B, am)
        if px:  # g3 as PX planes for the conv3 dgrad and weight gradient
            am.px[EX_G3] = True
            g3 = torch.empty((B, 7, 7, 128), dtype=torch.int16, device=df.device)
        else:
            g3 = torch.empty((B, 7, 7, 64), device=df.device)
        ps = isinstance(am, PassState)
        pdf = dfp is not None and ps and am.px[EX_DF]
        native.nature_fc_dgrad(dfp if pdf else df.contiguous(), B, self.qfc[1], h3 if not (ps and am.px[EX_H3]) else None,
                               g3, amax_df=am[AM_DF], amax_g3=am[AM_G3], relu_bits=am.bits[2] if ps else None,
                               g3_exp=am.exp(EX_G3) if px else None, df_exp=am.exp(EX_DF) if pdf else None)
        return g3

    def backward_acts(self, x, h1, h2, h3, dh3, dw1, db1, dw2, db2, dw3, db3, g3=None, am=None):
        """Trunk backward from dL/dh3 (f32 math: B x 3136 in NCHW order, before the ReLU mask)
        — or from g3, the already masked NHWC grad whose amax is in am[AM_G3] (am: the forward
        pass's table): writes (overwrites) the six conv gradients."""
        B = x.shape[0]
        if B == 0:
            for t in (dw1, db1, dw2, db2, dw3, db3):
                t.zero_()
            return
        dev = x.device
        if g3 is None:
            g3 = torch.empty((B, 7, 7, 64), device=dev)
            native.nchw_to_nhwc_relu_grad(dh3, h3, B, g3)      # ReLU backward of conv3, to NHWC
            if self.math != "f32":
                native.amax(g3, am[AM_G3])
        side = side_stream(dev) if BWD_STREAMS and dev.type == "cuda" else None
        cur = current_stream(dev) if side is not None else None
        if side is not None:  # wgrad3 beside dgrad3 (the tensors stay referenced until the join below)
            fork(side, cur)
        self.wgrad(3, h2, B, g3, dw3, db3, am, stream=side)
        if self.px_g2(B, am):  # g2 as PX planes for the direct conv2 dgrad and the conv2 weight gradient
            am.px[EX_G2] = True
            g2 = torch.empty((B, 9, 9, 128), dtype=torch.int16, device=dev)
        else:
            g2 = torch.empty((B, 9, 9, 64), device=dev)
        self.dgrad(3, g3, B, h2, g2, am)                        # dX of conv3, times ReLU'(conv2)
        if self._diag is not None:  # (tests: the pass's backward intermediates)
            self._diag.update(g3=g3, g2=g2, am=am)
        # wgrad2 beside the conv2 dgrad below BWD_SOLO_DGRAD2_BATCH rows (PPOX_BWD_SOLO_DGRAD2; default: every
        # batch); from it, the persistent conv2 dgrad runs alone — the side stream drained before it, wgrad2
        # forked after it, beside wgrad1.  Round 4 measured the two the same at 16,384 rows; with the direct
        # conv2 dgrad (round 5) the solo form idles the main stream ~150 µs while the side stream finishes the
        # conv3 weight gradient: 556.4 / 557.8k vs 560.8 / 559.2k env-steps/s (profiles/r05i)
        solo = side is not None and B >= BWD_SOLO_DGRAD2_BATCH
        late = None
        if side is not None and not solo:
            if FORK_LATE:  # the fork point recorded now, the side stream's wait issued after the dgrad
                late = _event(side, 2)
                late.record(cur)
            else:
                fork(side, cur)
                self.wgrad(2, h1, B, g2, dw2, db2, am, stream=side)
        if solo:
            join(side, cur)
        g1 = torch.empty((B, 20, 20, 32), device=dev)
        self.dgrad(2, g2, B, h1 if not self.h1p else None, g1, am)                        # dX of conv2, times ReLU'(conv1)
        if self._diag is not None:
            self._diag["g1"] = g1
        if late is not None:
            side.wait_event(late)
            self.wgrad(2, h1, B, g2, dw2, db2, am, stream=side)
        if side is None or (solo and BWD_SOLO_WGRAD2):
            self.wgrad(2, h1, B, g2, dw2, db2, am)
        elif solo:
            fork(side, cur)
            self.wgrad(2, h1, B, g2, dw2, db2, am, stream=side)
        self.wgrad(1, x, B, g1, dw1, db1, am)
        if side is not None:
            join(side, cur)

    def __call__(self, x):
        if x.dtype != torch.uint8:
            raise TypeError("NatureCNN trunk expects uint8 frame stacks (N, 4, 84, 84)")
        x = x.contiguous()
        return _NatureTrunk.apply(x, self, self.c1.weight, self.c1.bias, self.c2.weight, self.c2.bias,
                                  self.c3.weight, self.c3.bias)


def attach(net, flat, math=None):
    """Route a CnnActorCritic's convolutions through libppox."""
    net.conv_impl = NatureConvs(net, flat, math)
    return net.conv_impl
