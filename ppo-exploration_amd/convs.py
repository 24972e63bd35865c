"""NatureCNN conv trunk on the libppox MFMA implicit-GEMM kernels.

Forward: ppox_nature_conv_fwd (fp32 MFMA, fused u8->f32, bias, ReLU) for the
three convolutions of .ipynb_checkpoints/models-checkpoint.py:52-58, with
activations laid out NHWC between layers and NCHW at the trunk output (the
reference's Flatten order for Linear(3136, 512)).
Backward: libppox dgrad/wgrad kernels when present, else the ROCm library path
(aten.convolution_backward) on the same tensors — forward never falls back.
"""
import torch

import native


class _NatureTrunk(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, convs, w1, b1, w2, b2, w3, b3):
        convs.pack()
        B = x.shape[0]
        dev = x.device
        h1 = torch.empty((B, 20, 20, 32), device=dev)
        h2 = torch.empty((B, 9, 9, 64), device=dev)
        h3 = torch.empty((B, 64, 7, 7), device=dev)
        if B:
            native.nature_conv_fwd(1, x, B, None, 0, 0, 4 * 84 * 84, convs.wp1, b1, h1)
            native.nature_conv_fwd(2, h1, B, None, 0, 0, 0, convs.wp2, b2, h2)
            native.nature_conv_fwd(3, h2, B, None, 0, 0, 0, convs.wp3, b3, h3)
        ctx.save_for_backward(x, h1, h2, h3, w1, w2, w3)
        return h3

    @staticmethod
    def backward(ctx, dh3):
        x, h1, h2, h3, w1, w2, w3 = ctx.saved_tensors
        conv_bwd = torch.ops.aten.convolution_backward
        g3 = dh3 * (h3 > 0)
        h2c = h2.permute(0, 3, 1, 2)  # NCHW view, channels_last storage
        dh2, dw3, db3 = conv_bwd(g3, h2c, w3, [64], [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [True, True, True])
        g2 = dh2 * (h2c > 0)
        h1c = h1.permute(0, 3, 1, 2)
        dh1, dw2, db2 = conv_bwd(g2, h1c, w2, [64], [2, 2], [0, 0], [1, 1], False, [0, 0], 1, [True, True, True])
        g1 = dh1 * (h1c > 0)
        _, dw1, db1 = conv_bwd(g1, x.float(), w1, [32], [4, 4], [0, 0], [1, 1], False, [0, 0], 1,
                               [False, True, True])
        return None, None, dw1, db1, dw2, db2, dw3, db3


class NatureConvs:
    """Callable conv trunk bound to a CnnActorCritic whose parameters live in a FlatParams."""

    def __init__(self, net, flat):
        fe = net.feature_extractor
        self.c1, self.c2, self.c3 = fe[0], fe[2], fe[4]
        self.flat = flat
        dev = flat.device
        self.wp1 = torch.empty(256 * 32, device=dev)
        self.wp2 = torch.empty(512 * 64, device=dev)
        self.wp3 = torch.empty(576 * 64, device=dev)
        self._version = None

    def pack(self):
        v = (self.flat.step_count, self.flat.data.data_ptr())
        if v != self._version:
            native.nature_pack_weights(self.c1.weight, self.c2.weight, self.c3.weight, self.wp1, self.wp2, self.wp3)
            self._version = v

    def invalidate(self):
        self._version = None

    def __call__(self, x):
        if x.dtype != torch.uint8:
            raise TypeError("NatureCNN trunk expects uint8 frame stacks (N, 4, 84, 84)")
        x = x.contiguous()
        return _NatureTrunk.apply(x, self, self.c1.weight, self.c1.bias, self.c2.weight, self.c2.bias,
                                  self.c3.weight, self.c3.bias)


def attach(net, flat):
    """Route a CnnActorCritic's convolutions through libppox."""
    net.conv_impl = NatureConvs(net, flat)
    return net.conv_impl
