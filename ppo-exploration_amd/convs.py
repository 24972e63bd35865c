"""NatureCNN conv trunk on the libppox MFMA implicit-GEMM kernels.

Forward: ppox_nature_conv_fwd (fp32 MFMA, fused u8->f32, bias, ReLU) for the
three convolutions of .ipynb_checkpoints/models-checkpoint.py:52-58, with
activations laid out NHWC between layers and NCHW at the trunk output (the
reference's Flatten order for Linear(3136, 512)).
Backward: libppox MFMA dgrad (ReLU backward of the layer below fused) and
split-K wgrad (+ bias grad, deterministic fixed-order reduction) kernels.
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
        ctx.convs = convs
        ctx.save_for_backward(x, h1, h2, h3)
        return h3

    @staticmethod
    def backward(ctx, dh3):
        x, h1, h2, h3 = ctx.saved_tensors
        convs = ctx.convs
        B = x.shape[0]
        dev = x.device
        grads = [torch.zeros_like(t) for t in (convs.c1.weight, convs.c1.bias, convs.c2.weight, convs.c2.bias,
                                               convs.c3.weight, convs.c3.bias)]
        if B == 0:
            return (None, None, *grads)
        dw1, db1, dw2, db2, dw3, db3 = grads
        dh3 = dh3.contiguous()
        g3 = torch.empty((B, 7, 7, 64), device=dev)
        native.nchw_to_nhwc_relu_grad(dh3, h3, B, g3)          # ReLU backward of conv3, to NHWC
        native.nature_conv_wgrad(3, h2, B, None, 0, 0, 0, g3, convs.workspace(3, B), dw3, db3)
        g2 = torch.empty((B, 9, 9, 64), device=dev)
        native.nature_conv_dgrad(3, g3, B, convs.wpd3, h2, g2)  # dX of conv3, times ReLU'(conv2)
        native.nature_conv_wgrad(2, h1, B, None, 0, 0, 0, g2, convs.workspace(2, B), dw2, db2)
        g1 = torch.empty((B, 20, 20, 32), device=dev)
        native.nature_conv_dgrad(2, g2, B, convs.wpd2, h1, g1)  # dX of conv2, times ReLU'(conv1)
        native.nature_conv_wgrad(1, x, B, None, 0, 0, 4 * 84 * 84, g1, convs.workspace(1, B), dw1, db1)
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
        self.wpd2 = torch.empty(4 * 256 * 32, device=dev)
        self.wpd3 = torch.empty(576 * 64, device=dev)
        self._ws = {}
        self._version = None

    def workspace(self, layer, batch):
        need = native.nature_wgrad_workspace_bytes(layer, batch)
        ws = self._ws.get(layer)
        if ws is None or ws.numel() < need:
            ws = torch.empty(need, dtype=torch.uint8, device=self.flat.device)
            self._ws[layer] = ws
        return ws

    def pack(self):
        v = (self.flat.step_count, self.flat.data.data_ptr())
        if v != self._version:
            native.nature_pack_weights(self.c1.weight, self.c2.weight, self.c3.weight, self.wp1, self.wp2, self.wp3,
                                       self.wpd2, self.wpd3)
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
