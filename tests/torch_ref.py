"""Plain PyTorch fp64 CPU references of the Keras layer semantics used by the
per-kernel numerics tests (Keras NHWC/HWIO conventions, TF 'same' padding).
Test infrastructure only."""
import torch
import torch.nn.functional as F


def conv2d_ref(x, w, stride, pads, bias=None):
    """x NHWC, w HWIO [kh,kw,Ci,Co], pads (t,b,l,r) -> NHWC."""
    xt = x.permute(0, 3, 1, 2)
    pt, pb, pl, pr = pads
    xt = F.pad(xt, (pl, pr, pt, pb))
    y = F.conv2d(xt, w.permute(3, 2, 0, 1).contiguous(), bias=bias, stride=stride)
    return y.permute(0, 2, 3, 1)


def conv2d_transpose_ref(x, w, stride, pads, out_hw, bias=None):
    """Keras Conv2DTranspose: x NHWC [N,H,W,Cin], w [kh,kw,F,Cin]; pads of the equivalent conv."""
    xt = x.permute(0, 3, 1, 2)
    y = F.conv_transpose2d(xt, w.permute(3, 2, 0, 1).contiguous(), stride=stride)
    pt, pb, pl, pr = pads
    Ho, Wo = out_hw
    y = y[:, :, pt:pt + Ho, pl:pl + Wo]
    if bias is not None:
        y = y + bias.view(1, -1, 1, 1)
    return y.permute(0, 2, 3, 1)
