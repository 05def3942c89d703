"""CPU restatement of the reference network and train step (TEST INFRASTRUCTURE — oracle).

This is the checker for the HIP path, never the product: only tests/,
__graft_entry__.smoke() and bench.py's `cpu_baseline` leg may import it.

A functional torch-eager (CPU, fp32 or fp64) restatement of
/root/reference/model/segment.py, written against a flat parameter dict keyed by
the reference's state_dict names. Every block cites the reference lines it follows.
It is pinned against golden vectors produced by the reference module itself
(tests/golden/make_golden.py -> tests/golden/*.npz, see tests/test_oracle_golden.py).

Semantics kept from the reference:
  * `Conv` = conv2d(bias=True) -> BatchNorm2d(eps 1e-5, momentum 0.1) -> act
    (segment.py:34-45); act None -> identity (:42)
  * train-mode BN uses biased batch variance, updates running stats with the
    unbiased one and bumps num_batches_tracked (torch BatchNorm2d semantics)
  * `BottleneckDim_Res(usePrelu=False)` still uses PReLU inside (:174-188)
  * BCELoss clamps log at -100 (torch semantics) and is applied to sigmoid(logits)
    (train_instance.py:299,377-378; segment.py:531-534)
  * Adam defaults lr 1e-3, betas (0.9, 0.999), eps 1e-8 (train_instance.py:297)
"""
import torch
import torch.nn.functional as F

BN_EPS = 1e-5
BN_MOMENTUM = 0.1


class Ctx:
    def __init__(self, params, train):
        self.P = params          # dict key -> tensor (parameters and buffers)
        self.train = train

    def __getitem__(self, k):
        return self.P[k]


def _bn(c, pre, x):
    """BatchNorm2d (segment.py:41, :306-307)."""
    P = c.P
    w, b = P[pre + ".weight"], P[pre + ".bias"]
    rm, rv = P[pre + ".running_mean"], P[pre + ".running_var"]
    if c.train:
        with torch.no_grad():
            P[pre + ".num_batches_tracked"] += 1
        # F.batch_norm updates rm/rv in place with the unbiased variance
        return F.batch_norm(x, rm, rv, w, b, training=True, momentum=BN_MOMENTUM, eps=BN_EPS)
    return F.batch_norm(x, rm, rv, w, b, training=False, eps=BN_EPS)


def _act(c, pre, kind, x):
    if kind == "prelu":
        return F.prelu(x, c.P[pre + ".weight"])
    if kind == "relu":
        return F.relu(x)
    return x


def conv(c, pre, x, k=1, s=1, p=None, g=1, d=1, act=None):
    """`Conv` (segment.py:34-45) with `autopad` (:12-16)."""
    if p is None:
        p = k // 2 if isinstance(k, int) else tuple(v // 2 for v in k)
    y = F.conv2d(x, c.P[pre + ".conv.weight"], c.P[pre + ".conv.bias"], stride=s,
                 padding=p, dilation=d, groups=g)
    y = _bn(c, pre + ".bn", y)
    return _act(c, pre + ".act", act, y)


def init_head_s4(c, pre, x):
    """segment.py:19-31: cat(maxpool4(x), Conv5x5s2(Conv5x5s2(x)))."""
    short = F.max_pool2d(x, kernel_size=4, stride=4)
    y = conv(c, pre + ".layer1", x, k=5, s=2, p=2, act="prelu")
    y = conv(c, pre + ".layer2", y, k=5, s=2, p=2, act="prelu")
    return torch.cat((short, y), 1)


def bottleneck3x3(c, pre, x, planes, pad=1, dil=1):
    """segment.py:52-79."""
    y = conv(c, pre + ".convs.0", x, k=1, act="prelu")
    y = conv(c, pre + ".convs.1", y, k=3, p=pad, d=dil, g=planes, act="prelu")
    y = conv(c, pre + ".convs.2", y, k=1, act=None)
    return F.prelu(y + x, c.P[pre + ".prelu.weight"])


def bottleneck5x5(c, pre, x, planes):
    """segment.py:82-111 — bare depthwise (5,1) conv with bias, no BN/act (:91-92)."""
    y = conv(c, pre + ".convs.0", x, k=1, act="prelu")
    y = F.conv2d(y, c.P[pre + ".convs.1.weight"], c.P[pre + ".convs.1.bias"],
                 padding=(2, 0), groups=planes)
    y = conv(c, pre + ".convs.2", y, k=(1, 5), p=(0, 2), g=planes, act="prelu")
    y = conv(c, pre + ".convs.3", y, k=1, act=None)
    return F.prelu(y + x, c.P[pre + ".prelu.weight"])


def bottleneck_down2(c, pre, x, planes):
    """segment.py:114-150; returns (out, maxpool2(x))."""
    y = conv(c, pre + ".convs.0", x, k=2, s=2, p=0, act="prelu")
    y = conv(c, pre + ".convs.1", y, k=3, s=1, p=1, g=planes, act="prelu")
    y = conv(c, pre + ".convs.2", y, k=1, act=None)
    r1 = F.max_pool2d(x, kernel_size=2, stride=2)
    r = conv(c, pre + ".convm.0", r1, k=1, act=None)
    return F.prelu(y + r, c.P[pre + ".prelu.weight"]), r1


def bottleneck_dim_res(c, pre, x, planes, use_prelu):
    """segment.py:153-209 — inner acts are PReLU in both branches (:162-183)."""
    y = conv(c, pre + ".convs.0", x, k=1, act="prelu")
    y = conv(c, pre + ".convs.1", y, k=3, p=1, g=planes, act="prelu")
    y = conv(c, pre + ".convs.2", y, k=1, act=None)
    y = y + conv(c, pre + ".resconv.0", x, k=1, act=None)
    return F.prelu(y, c.P[pre + ".prelu.weight"]) if use_prelu else F.relu(y)


def bottleneck_dim_relu(c, pre, x):
    """segment.py:212-261, usePrelu=False path: dense 3x3 + ReLU (:233-247)."""
    y = conv(c, pre + ".convs.0", x, k=1, act="relu")
    y = conv(c, pre + ".convs.1", y, k=3, p=1, act="relu")
    y = conv(c, pre + ".convs.2", y, k=1, act=None)
    return F.relu(y + x)


def bottleneck_up_res(c, pre, x, skip):
    """segment.py:296-335 (and _Other :338-344): convT k4 s2 p1 + BN + ReLU branch,
    residual = 1x1(up2(cat(1x1(x), skip)))."""
    P = c.P
    y = conv(c, pre + ".convs.0", x, k=1, act="relu")
    y = F.conv_transpose2d(y, P[pre + ".convs.1.weight"], P[pre + ".convs.1.bias"],
                           stride=2, padding=1)
    y = F.relu(_bn(c, pre + ".convs.2", y))                 # convs.3 is nn.ReLU (:308)
    y = conv(c, pre + ".convs.4", y, k=1, act=None)
    r = conv(c, pre + ".conv2.0", x, k=1, act=None)
    r = F.interpolate(torch.cat([r, skip], 1), scale_factor=2, mode="nearest")
    r = F.conv2d(r, P[pre + ".uppool.1.weight"], P[pre + ".uppool.1.bias"])
    return F.relu(y + r)


def segment_forward(c, x):
    """`Segment.forward` (segment.py:466-508): logits [N,1,H,W]."""
    init_down = init_head_s4(c, "init_conv", x)                              # :472
    b1_down, b1_idx = bottleneck_down2(c, "bottle1_1", init_down, 16)        # :478
    y = b1_down
    for i in range(4):                                                       # :479, :366-375
        y = bottleneck3x3(c, f"bottle1_x.{i}", y, 16)
    b2_down, b2_idx = bottleneck_down2(c, "bottle2_1", y, 16)                # :482
    y = _section_x(c, "bottle2_x", b2_down)                                  # :483, :382-396
    y = bottleneck_dim_res(c, "bottle3_1", torch.cat((y, b2_down), 1), 48, True)  # :485-488
    y = _section_x(c, "bottle3_x", y)                                        # :489, :402-417
    b4_1 = bottleneck_up_res(c, "bottle4_1up", y, b2_idx)                    # :492
    y = bottleneck_dim_res(c, "bottle4_2", torch.cat((b1_down, b4_1), 1), 16, False)  # :494-496
    y = bottleneck_dim_relu(c, "bottle4_3", y)                               # :497
    y = bottleneck_up_res(c, "bottle5_1up", y, b1_idx)                       # :500
    y = bottleneck_dim_relu(c, "bottle5_2", y)                               # :501
    y = F.conv_transpose2d(y, c.P["bottle6_1.weight"], c.P["bottle6_1.bias"],
                           stride=4, padding=2)                              # :504, :435-436
    return F.conv2d(y, c.P["bottle6_2.weight"], c.P["bottle6_2.bias"], padding=1)  # :505


def _section_x(c, pre, y):
    """Bottleneck3x3 d1, d2, d1, d4, then Bottleneck5x5 (segment.py:382-396)."""
    for i, dil in enumerate((1, 2, 1, 4)):
        y = bottleneck3x3(c, f"{pre}.{i}", y, 48, pad=dil, dil=dil)
    return bottleneck5x5(c, f"{pre}.4", y, 48)


def bce_loss(prob, target):
    """nn.BCELoss() mean reduction (train_instance.py:299,378), log clamped at -100."""
    return F.binary_cross_entropy(prob, target)


def train_step(params, x, target, dtype=torch.float64):
    """One reference train step body (train_instance.py:375-379) minus the optimizer:
    returns (logits, loss, grads-by-key). `params` (key -> tensor) is updated in place
    for BN running stats."""
    P = {}
    for k, v in params.items():
        t = torch.as_tensor(v)
        P[k] = t.to(dtype) if t.is_floating_point() else t.clone()
        if k.endswith(("weight", "bias")) and not k.endswith(("running_mean", "running_var")):
            P[k].requires_grad_(True)
    c = Ctx(P, train=True)
    xt = torch.as_tensor(x).to(dtype)
    logits = segment_forward(c, xt)
    prob = torch.sigmoid(logits)                                             # segment.py:534
    loss = bce_loss(prob, torch.as_tensor(target).to(dtype))
    loss.backward()
    grads = {k: (t.grad.detach().clone() if t.grad is not None else None)
             for k, t in P.items() if t.requires_grad}
    return logits.detach(), loss.detach(), grads, P


def forward(params, x, train=False, dtype=torch.float64):
    P = {k: (torch.as_tensor(v).to(dtype) if torch.as_tensor(v).is_floating_point()
             else torch.as_tensor(v).clone()) for k, v in params.items()}
    with torch.no_grad():
        logits = segment_forward(Ctx(P, train), torch.as_tensor(x).to(dtype))
    return logits, P


def adam_step(param, grad, exp_avg, exp_avg_sq, step, lr=1e-3, beta1=0.9, beta2=0.999,
              eps=1e-8):
    """torch.optim.Adam default update (train_instance.py:297,380), single tensor.
    step is the 1-based step count after increment. Updates arrays in place."""
    exp_avg.mul_(beta1).add_(grad, alpha=1 - beta1)
    exp_avg_sq.mul_(beta2).addcmul_(grad, grad, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = (exp_avg_sq.sqrt() / (bc2 ** 0.5)).add_(eps)
    param.addcdiv_(exp_avg, denom, value=-(lr / bc1))
    return param
