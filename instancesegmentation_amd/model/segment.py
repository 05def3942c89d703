"""Drop-in replacement for the reference `model/segment.py` (`from model.segment import
Segment`, train_instance.py:23).

Same classes, constructor signatures, attribute names, parameter order and
state_dict keys (588 entries for Segment(20)), so reference checkpoints and
`optim.Adam(model.parameters())` (train_instance.py:297) keep working. What changes
is `forward`: each module's structure is described once in `emit` and executed by
the MI355X engine (instancesegmentation_amd/engine.py -> libisg.so HIP kernels),
not by torch eager kernels. There is no CPU path: a CPU tensor raises.

Reference anchors: Conv :34-48, init_head_s4 :19-31, Bottleneck3x3 :52-79,
Bottleneck5x5 :82-111, BottleneckDown2 :114-150, BottleneckDim_Res :153-209,
BottleneckDim :212-261, BottleneckUp (dead code) :264-293, BottleneckUp_Res :296-335,
BottleneckUp_Res_Other :338-344, Segment :347-534.
"""
import torch
import torch.nn as nn

from ..engine import Keypoints, Val, Value, cat
from ..runtime import EngineModule, sigmoid


def autopad(k, p=None):
    """segment.py:12-16 — 'same' padding for odd kernels."""
    if p is None:
        p = k // 2 if isinstance(k, int) else [x // 2 for x in k]
    return p


class Conv(EngineModule):
    """conv2d(bias) -> BatchNorm2d -> act (segment.py:34-45)."""

    def __init__(self, c1, c2, k=1, s=1, p=None, g=1, d=1, act=nn.Hardswish(), bias=True):
        super().__init__()
        self.conv = nn.Conv2d(c1, c2, k, s, autopad(k, p), groups=g, dilation=d, bias=bias)
        self.bn = nn.BatchNorm2d(c2)
        self.act = act if act else nn.Identity()

    def emit(self, g, x, kp=None):
        kind, slope = g.act_of(self.act)
        return g.conv(self.conv, x, bn=getattr(self, "bn", None), act=kind, slope=slope,
                      name=g.mod_names.get(id(self), "conv"), kp=kp)

    def fuseforward(self, x):
        """segment.py:47-48 (BN already folded into conv): act(conv(x)). The traced
        plan is cached on the module (one trace per input shape)."""
        ff = self.__dict__.get("_ff")
        if ff is None:
            ff = _FuseForward(self)
            object.__setattr__(self, "_ff", ff)  # not a submodule: no state_dict keys
        return ff(x)

    def fuse_(self):
        """Fold the BatchNorm (eval statistics) into the conv weights and bias and drop
        it, the yolov5-style fusion `fuseforward` presumes (segment.py:47-48):
        W' = W * g/sqrt(v+eps) per output channel, b' = (b - m) * g/sqrt(v+eps) + beta."""
        bn = getattr(self, "bn", None)
        if bn is None:
            return self
        fold_bn_(self.conv, bn, transposed=False)
        del self.bn
        self._plans.clear()
        return self


@torch.no_grad()
def fold_bn_(conv, bn, transposed):
    """Fold an eval-mode BatchNorm2d into the preceding (transposed) conv, in place, in
    double precision. Output channels: dim 0 of a Conv2d weight, dim 1 of a
    ConvTranspose2d weight."""
    scale = bn.weight.double() / torch.sqrt(bn.running_var.double() + bn.eps)
    w = conv.weight.double()
    shape = [1] * w.dim()
    shape[1 if transposed else 0] = -1
    conv.weight.copy_((w * scale.view(shape)).to(conv.weight.dtype))
    b = conv.bias.double() if conv.bias is not None else torch.zeros_like(scale)
    nb = (b - bn.running_mean.double()) * scale + bn.bias.double()
    if conv.bias is None:
        conv.bias = nn.Parameter(nb.to(conv.weight.dtype))
    else:
        conv.bias.copy_(nb.to(conv.bias.dtype))


class _FuseForward(EngineModule):
    def __init__(self, c):
        super().__init__()
        self.c = c

    def emit(self, g, x):
        kind, slope = g.act_of(self.c.act)
        return g.conv(self.c.conv, x, act=kind, slope=slope, name="fused")


class init_head_s4(EngineModule):
    """segment.py:19-31: cat(maxpool4(x), Conv5x5s2(PReLU) o Conv5x5s2(PReLU))."""

    def __init__(self, inplanes, planes, outplanes):
        super().__init__()
        self.layer1 = Conv(inplanes, planes, k=5, s=2, p=2, act=nn.PReLU(planes))
        self.layer2 = Conv(planes, outplanes - inplanes, k=5, s=2, p=2,
                           act=nn.PReLU(outplanes - inplanes))

    def emit(self, g, x, kp=None):
        """kp (engine.Keypoints): the input is cat(x, heatmaps of kp) with the heatmaps
        synthesised inside the stem kernels — same values, never in HBM."""
        cin = x.C + (kp.nparts if kp is not None else 0)
        cout = self.layer2.conv.out_channels
        out = g.act_buf(cin + cout, x.H // 4, x.W // 4, "init_down")
        short = g.maxpool(x, 4, out=out, c0=0)
        if kp is not None:  # one segment over the pooled image and heatmap channels
            g.kp_pool(kp, 4, x.H, x.W, out, c0=x.C)
            short = Value([Val(out, 0, cin, grad=short.grad)])
        y = self.layer2.emit(g, self.layer1.emit(g, x, kp=kp))
        y = g.materialize(y, out=out, c0=cin)
        return cat(short, y)


def _chain(g, seq, x):
    for m in seq:
        x = m.emit(g, x)
    return x


def _act_kind(g, mod):
    return g.act_of(mod)


class Bottleneck3x3(EngineModule):
    """segment.py:52-79: PReLU(x + 1x1(dw3x3_d(1x1(x))))."""

    def __init__(self, inplanes, planes, pad=1, dilation=1):
        super().__init__()
        self.convs = nn.Sequential(
            Conv(inplanes, planes, k=1, act=nn.PReLU(planes)),
            Conv(planes, planes, k=3, p=pad, d=dilation, g=planes, act=nn.PReLU(planes)),
            Conv(planes, inplanes, k=1, act=None),
        )
        self.prelu = nn.PReLU(inplanes)

    def emit(self, g, x):
        y = _chain(g, self.convs, x)
        kind, slope = g.act_of(self.prelu)
        return g.tail([(y, False), (x, False)], kind, slope, name=g.mod_names[id(self)])


class Bottleneck5x5(EngineModule):
    """segment.py:82-111; the (5,1) depthwise conv has bias and no BN/act (:91-92)."""

    def __init__(self, inplanes, planes):
        super().__init__()
        self.convs = nn.Sequential(
            Conv(inplanes, planes, k=1, act=nn.PReLU(planes)),
            nn.Conv2d(planes, planes, kernel_size=(5, 1), padding=(2, 0), groups=planes),
            Conv(planes, planes, k=(1, 5), p=(0, 2), g=planes, act=nn.PReLU(planes)),
            Conv(planes, inplanes, k=1, act=None),
        )
        self.prelu = nn.PReLU(inplanes)

    def emit(self, g, x):
        y = self.convs[0].emit(g, x)
        y = g.conv(self.convs[1], y, name=g.mod_names[id(self)] + ".dw51")
        y = self.convs[2].emit(g, y)
        y = self.convs[3].emit(g, y)
        kind, slope = g.act_of(self.prelu)
        return g.tail([(y, False), (x, False)], kind, slope, name=g.mod_names[id(self)])


class BottleneckDown2(EngineModule):
    """segment.py:114-150: returns (PReLU(convs(x) + convm(maxpool2(x))), maxpool2(x))."""

    def __init__(self, inplanes, planes, outplanes):
        super().__init__()
        self.convs = nn.Sequential(
            Conv(inplanes, planes, k=2, s=2, p=0, act=nn.PReLU(planes)),
            Conv(planes, planes, k=3, s=1, p=1, g=planes, act=nn.PReLU(planes)),
            Conv(planes, outplanes, k=1, act=None),
        )
        self.convm = nn.Sequential(Conv(inplanes, outplanes, k=1, act=None))
        self.prelu = nn.PReLU(outplanes)

    def emit(self, g, x):
        name = g.mod_names[id(self)]
        with g.side_branch():  # forward: overlaps the convs chain (engine._fork_branches)
            r1 = g.maxpool(x, 2, name=name + ".pool")
            r = self.convm[0].emit(g, r1)
        y = _chain(g, self.convs, x)
        kind, slope = g.act_of(self.prelu)
        return g.tail([(y, False), (r, False)], kind, slope, name=name), r1


class BottleneckDim_Res(EngineModule):
    """segment.py:153-209; with usePrelu=False the inner acts are STILL PReLU (:174-188)
    and only the final activation is ReLU."""

    def __init__(self, inplanes, planes, outplanes, usePrelu):
        super().__init__()
        self.usePrelu = usePrelu
        self.convs = nn.Sequential(
            Conv(inplanes, planes, k=1, act=nn.PReLU(planes)),
            Conv(planes, planes, k=3, p=1, g=planes, act=nn.PReLU(planes)),
            Conv(planes, outplanes, k=1, act=None),
        )
        self.resconv = nn.Sequential(Conv(inplanes, outplanes, k=1, act=None))
        self.prelu = nn.PReLU(outplanes)
        self.relu = nn.ReLU(inplace=True)

    def siblings(self):
        """The two 1x1 Convs reading x (engine.param_layout / Graph.conv_pair)."""
        return self.convs[0], self.resconv[0]

    def emit(self, g, x):
        pair = g.conv_pair(self.convs[0], self.resconv[0], x)  # one stacked GEMM
        if pair is not None:
            y0, r = pair
            y = _chain(g, self.convs[1:], y0)
        else:
            with g.side_branch():  # forward: overlaps the convs chain (engine._fork_branches)
                r = self.resconv[0].emit(g, x)
            y = _chain(g, self.convs, x)
        kind, slope = g.act_of(self.prelu if self.usePrelu else self.relu)
        return g.tail([(y, False), (r, False)], kind, slope, name=g.mod_names[id(self)])


class BottleneckDim(EngineModule):
    """segment.py:212-261 (usePrelu=False: 1x1+ReLU -> dense 3x3+ReLU -> 1x1, + x, ReLU)."""

    def __init__(self, inplanes, planes, outplanes, usePrelu):
        super().__init__()
        self.usePrelu = usePrelu
        if self.usePrelu:
            self.convs = nn.Sequential(
                Conv(inplanes, planes, k=1, act=nn.PReLU(planes)),
                Conv(planes, planes, k=3, p=1, g=planes, act=nn.PReLU(planes)),
                Conv(planes, outplanes, k=1, act=None),
            )
        else:
            self.convs = nn.Sequential(
                Conv(inplanes, planes, k=1, act=nn.ReLU(inplace=True)),
                Conv(planes, planes, k=3, p=1, act=nn.ReLU(inplace=True)),
                Conv(planes, outplanes, k=1, act=None),
            )
        self.prelu = nn.PReLU(outplanes)
        self.relu = nn.ReLU(inplace=True)

    def emit(self, g, x):
        y = _chain(g, self.convs, x)
        kind, slope = g.act_of(self.prelu if self.usePrelu else self.relu)
        return g.tail([(y, False), (x, False)], kind, slope, name=g.mod_names[id(self)])


class BottleneckUp(EngineModule):
    """segment.py:264-293 — never instantiated by the reference (MaxUnpool2d path); kept
    for import compatibility only."""

    def __init__(self, inplanes, planes, outplanes):
        super().__init__()
        self.convs = nn.Sequential(
            Conv(inplanes, planes, k=1, act=nn.ReLU(inplace=True)),
            nn.ConvTranspose2d(planes, planes, kernel_size=4, padding=1, stride=2),
            nn.BatchNorm2d(planes),
            nn.ReLU(inplace=True),
            Conv(planes, outplanes, k=1, act=None),
        )
        self.conv2 = nn.Conv2d(inplanes, outplanes, kernel_size=1)
        self.uppool = nn.MaxUnpool2d(2, stride=2)

    def emit(self, g, x, mp_indices):
        raise NotImplementedError("BottleneckUp (MaxUnpool2d) is dead code in the reference "
                                  "(segment.py:264-293) and not on the MI355X hot path")


class BottleneckUp_Res(EngineModule):
    """segment.py:296-335. relu(convs(x) + 1x1(up2(cat(conv2(x), skip)))). The 1x1 conv of
    `uppool` is applied before the nearest x2 upsample (exactly equal per pixel, 4x less
    work); the tail reads it at half resolution."""

    def __init__(self, inplanes, planes, outplanes):
        super().__init__()
        self.convs = nn.Sequential(
            Conv(inplanes, planes, k=1, act=nn.ReLU(inplace=True)),
            nn.ConvTranspose2d(planes, planes, kernel_size=4, padding=1, stride=2),
            nn.BatchNorm2d(planes),
            nn.ReLU(inplace=True),
            Conv(planes, outplanes, k=1, act=None),
        )
        self.conv2 = nn.Sequential(Conv(inplanes, outplanes, k=1, act=None))
        self.uppool = nn.Sequential(
            nn.UpsamplingNearest2d(scale_factor=2),
            nn.Conv2d(outplanes * 2, outplanes, 1, 1, 0),
        )

    def siblings(self):
        """The two 1x1 Convs reading x (engine.param_layout / Graph.conv_pair)."""
        return self.convs[0], self.conv2[0]

    def emit(self, g, x, mp_indices):
        name = g.mod_names[id(self)]
        up, c1 = self.uppool[0], self.uppool[1]
        if not (isinstance(up, nn.UpsamplingNearest2d) and up.scale_factor in (2, 2.0, (2, 2))
                and c1.kernel_size == (1, 1)):
            raise NotImplementedError("uppool must be nearest x2 followed by a 1x1 conv")
        pair = g.conv_pair(self.convs[0], self.conv2[0], x)  # one stacked GEMM
        if pair is not None:
            y, r = pair
            with g.side_branch():  # forward: overlaps the convT chain
                u = g.conv(c1, cat(r, mp_indices), name=name + ".uppool")
        else:
            with g.side_branch():  # forward: overlaps the convs chain (engine._fork_branches)
                r = self.conv2[0].emit(g, x)
                u = g.conv(c1, cat(r, mp_indices), name=name + ".uppool")
            y = self.convs[0].emit(g, x)
        kind, slope = g.act_of(self.convs[3])
        bn = self.convs[2] if isinstance(self.convs[2], nn.BatchNorm2d) else None
        y = g.conv_transpose(self.convs[1], y, bn=bn, act=kind, slope=slope,
                             name=name + ".convT")
        y = self.convs[4].emit(g, y)
        return g.tail([(y, False), (u, True)], "relu", None, name=name)


class BottleneckUp_Res_Other(BottleneckUp_Res):
    """segment.py:338-344 — skip connection with `other` channels."""

    def __init__(self, inplanes, planes, outplanes, other):
        super().__init__(inplanes, planes, outplanes)
        self.uppool = nn.Sequential(
            nn.UpsamplingNearest2d(scale_factor=2),
            nn.Conv2d(outplanes + other, outplanes, 1, 1, 0),
        )


class Segment(EngineModule):
    """segment.py:347-534. forward(x[N,C_in,H,W]) -> logits [N,1,H,W] (H, W multiples of
    16, as the reference requires — SURVEY.md §0.5); train_batch(x, heatmaps) ->
    sigmoid probabilities."""

    def __init__(self, in_channel):
        super().__init__()
        self.export = False
        self.output_mid_features = False

        self.init_Dim = 16 + in_channel
        self.init_conv = init_head_s4(in_channel, 16, self.init_Dim)

        self.bottle1_downDim = 16
        self.bottle1_Dim = 48
        self.bottle1_1 = BottleneckDown2(self.init_Dim, self.bottle1_downDim, self.bottle1_Dim)
        self.bottle1_x = nn.Sequential(
            *[Bottleneck3x3(self.bottle1_Dim, self.bottle1_downDim) for _ in range(4)])

        self.bottle2_downDim = 48
        self.bottle2_Dim = 128
        self.bottle2_1 = BottleneckDown2(self.bottle1_Dim, self.bottle1_downDim, self.bottle2_Dim)
        self.bottle2_x = self._section(self.bottle2_Dim, self.bottle2_downDim)

        self.bottle3_1 = BottleneckDim_Res(self.bottle2_Dim * 2, self.bottle2_downDim,
                                           self.bottle2_Dim, usePrelu=True)
        self.bottle3_x = self._section(self.bottle2_Dim, self.bottle2_downDim)

        self.bottle4_1up = BottleneckUp_Res(self.bottle2_Dim, self.bottle1_downDim, self.bottle1_Dim)
        self.bottle4_2 = BottleneckDim_Res(self.bottle1_Dim * 2, 16, self.bottle1_Dim,
                                           usePrelu=False)
        self.bottle4_3 = BottleneckDim(self.bottle1_Dim, 16, self.bottle1_Dim, usePrelu=False)

        self.bottle5_1up = BottleneckUp_Res_Other(self.bottle1_Dim, 4, self.bottle1_downDim,
                                                  self.init_Dim)
        self.bottle5_2 = BottleneckDim(self.bottle1_downDim, 4, self.bottle1_downDim, usePrelu=False)

        self.bottle6_1 = nn.ConvTranspose2d(self.bottle1_downDim, 4, kernel_size=8, padding=2,
                                            stride=4)
        self.bottle6_2 = nn.Conv2d(4, 1, kernel_size=3, padding=1)

        self.weights_init()

    @staticmethod
    def _section(dim, down):
        """Bottleneck3x3 d1, d2, d1, d4 + Bottleneck5x5 (segment.py:382-396, 402-417)."""
        return nn.Sequential(
            Bottleneck3x3(dim, down),
            Bottleneck3x3(dim, down, pad=2, dilation=2),
            Bottleneck3x3(dim, down),
            Bottleneck3x3(dim, down, pad=4, dilation=4),
            Bottleneck5x5(dim, down),
        )

    def weights_init(self):
        """segment.py:451-464: kaiming-normal(fan_in, relu) on nn.Conv2d only (ConvTranspose2d
        keeps torch's default init), zero conv bias, BN weight 1 / bias 0."""
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_in", nonlinearity="relu")
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, 0, 0.01)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)

    def emit(self, g, x, heatmaps=None):
        kp = None
        if isinstance(heatmaps, Keypoints):
            kp = heatmaps  # heatmaps synthesised from keypoints inside the stem
        elif heatmaps is not None:
            x = cat(x, heatmaps)                                       # segment.py:532
        if x.H % 16 or x.W % 16:
            raise RuntimeError(f"Segment needs H, W multiples of 16, got {x.H}x{x.W} "
                               "(the reference fails in torch.cat otherwise, SURVEY.md §0.5)")
        init_down = self.init_conv.emit(g, x, kp=kp)                   # :472
        b1_down, b1_idx = self.bottle1_1.emit(g, init_down)            # :478
        y = _chain(g, self.bottle1_x, b1_down)                         # :479
        b2_down, b2_idx = self.bottle2_1.emit(g, y)                    # :482
        y = _chain(g, self.bottle2_x, b2_down)                         # :483
        y = self.bottle3_1.emit(g, cat(y, b2_down))                    # :485-488
        y = _chain(g, self.bottle3_x, y)                               # :489
        b4_1 = self.bottle4_1up.emit(g, y, b2_idx)                     # :492
        y = self.bottle4_2.emit(g, cat(b1_down, b4_1))                 # :494-496
        y = self.bottle4_3.emit(g, y)                                  # :497
        y = self.bottle5_1up.emit(g, y, b1_idx)                        # :500
        y = self.bottle5_2.emit(g, y)                                  # :501
        head = g.head(self.bottle6_1, self.bottle6_2, y, name="logits")  # :504-505 fused
        if head is not None:
            return head
        y = g.conv_transpose(self.bottle6_1, y, name="bottle6_1")      # :504
        return g.conv(self.bottle6_2, y, name="logits")                # :505

    def fuse(self):
        """Inference form (Conv.fuseforward, segment.py:47-48): every BatchNorm folded
        into the conv / transposed conv in front of it, in place; the module stays in
        eval mode (the folded weights bake the running statistics in). Returns self."""
        self.eval()
        for m in list(self.modules()):
            if isinstance(m, Conv):
                m.fuse_()
            elif isinstance(m, BottleneckUp_Res) and isinstance(m.convs[2], nn.BatchNorm2d):
                fold_bn_(m.convs[1], m.convs[2], transposed=True)
                m.convs[2] = nn.Identity()
        self.clear_plans()
        for m in self.modules():
            if isinstance(m, EngineModule):
                m.clear_plans()
        self.fused = True
        return self

    def train(self, mode=True):
        if mode and getattr(self, "fused", False):
            raise RuntimeError("a fused Segment (BatchNorm folded) is inference-only")
        return super().train(mode)

    def train_batch(self, x, heatmaps):
        """segment.py:531-534: sigmoid(forward(cat([x, heatmaps], 1))); the concat is read
        in place by the first kernels (two input segments), not materialised. heatmaps may
        also be the keypoints they come from, float64 [N, 17, 3] = (x, y, visible)
        (train_instance.py:33-68): the maps are then synthesised inside the stem."""
        return sigmoid(self(x, heatmaps))
