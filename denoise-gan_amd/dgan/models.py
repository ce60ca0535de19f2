"""Keras-shaped network objects over the libdgan executors.

`Generator` / `Discriminator` reproduce what the reference's drivers and
inference scripts touch on a tf.keras.Model (train_pix2pix.py:44-48, :64-69,
:105, :158-161, :192-195; infer.py:40-55):
  net(x, training=...)           forward on the HIP path
  net.trainable_variables        device views into the flat parameter arena
  net.non_trainable_variables    BN moving statistics
  net.count_params(), net.summary(), net.save(path), net.load_weights(path),
  net.get_weights(), net.set_weights(list)
and `Adam` reproduces tf.keras.optimizers.Adam's apply_gradients /
iterations surface with TF ApplyAdam arithmetic (ops.adam).
"""
import json
import os

import numpy as np
import torch

from . import ops
from .nets import (Arena, BNState, DiscriminatorPlan, GeneratorPlan, _bn_channels, d_layout_order, d_variables,
                   g_layout_order, g_variables, init_variables)


def default_device():
    if not torch.cuda.is_available():
        raise ops.DGError("no HIP device visible: the dgan path runs only on the GPU (no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


def to_device(a, device):
    """numpy / torch (any device) -> contiguous fp32 device tensor (NHWC)."""
    if isinstance(a, torch.Tensor):
        t = a.to(device=device, dtype=torch.float32)
    else:
        t = torch.as_tensor(np.asarray(a, dtype=np.float32), device=device)
    return t.contiguous()


class Network:
    kind = "network"

    def __init__(self, name, var_list, layout, width, seed, device=None):
        self.name = name
        self.width = width
        self.device = device or default_device()
        self.arena = Arena(var_list, self.device, layout)
        self.bn = BNState(_bn_channels(var_list), self.device)
        self.arena.load(init_variables(var_list, seed))
        self._plans = {}

    # --- Keras surface ---------------------------------------------------
    @property
    def trainable_variables(self):
        return [self.arena.param(n) for n, _ in self.arena.var_list]

    @property
    def trainable_variable_names(self):
        return [f"{self.name}/{n}" for n, _ in self.arena.var_list]

    @property
    def non_trainable_variables(self):
        out = []
        for k in self.bn.mean:
            out += [self.bn.mean[k], self.bn.var[k]]
        return out

    @property
    def variables(self):
        return self.trainable_variables + self.non_trainable_variables

    def count_params(self):
        return self.arena.count + sum(int(t.numel()) for t in self.non_trainable_variables)

    def summary(self, print_fn=print):
        print_fn(f'Model: "{self.name}"')
        for n, s in self.arena.var_list:
            print_fn(f"  {n:<28s} {str(tuple(s)):<22s} {int(np.prod(s)):>12,d}")
        nt = sum(int(t.numel()) for t in self.non_trainable_variables)
        print_fn(f"Total params: {self.count_params():,d}")
        print_fn(f"Trainable params: {self.arena.count:,d}")
        print_fn(f"Non-trainable params: {nt:,d}")

    def get_weights(self):
        w = self.arena.export()
        bn = self.bn.export()
        return [w[n] for n, _ in self.arena.var_list] + [bn[k] for k in sorted(bn)]

    def set_weights(self, weights):
        names = [n for n, _ in self.arena.var_list]
        self.arena.load(dict(zip(names, weights[:len(names)])))
        bnk = sorted(self.bn.export())
        self.bn.load(dict(zip(bnk, weights[len(names):])))

    def state_dict(self):
        d = {f"{n}": v for n, v in self.arena.export().items()}
        d.update(self.bn.export())
        return d

    def load_state_dict(self, d):
        self.arena.load({n: d[n] for n, _ in self.arena.var_list if n in d})
        self.bn.load(d)

    def save(self, path):
        """Weights with Keras variable names (HWIO / [kh,kw,F,Cin] kernels)."""
        os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
        arrays = self.state_dict()
        np.savez(path if path.endswith(".npz") else path + ".npz", **arrays)
        with open((path[:-4] if path.endswith(".npz") else path) + ".json", "w") as f:
            json.dump({"model": self.kind, "name": self.name, "width": self.width}, f)

    def load_weights(self, path):
        p = path if path.endswith(".npz") else path + ".npz"
        with np.load(p, allow_pickle=False) as z:
            self.load_state_dict({k: z[k] for k in z.files})

    def _plan(self, key, factory):
        if key not in self._plans:
            self._plans[key] = factory()
        return self._plans[key]


class Generator(Network):
    """pix2pix U-Net generator (pix2pix.py:144-192)."""
    kind = "pix2pix_generator"

    def __init__(self, width=1, seed=1234, device=None):
        super().__init__("generator", g_variables(width), g_layout_order(width), width, seed, device)

    def __call__(self, x, training=False, drop_rate=0.5, drop_seed=0):
        x = to_device(x, self.device)
        N, H, W, _ = x.shape
        plan = self._plan(("fwd", N, H, W),
                          lambda: GeneratorPlan(N, H, W, self.width, self.arena, self.bn, self.device, 1, False))
        ws = ops.Workspace(self.device)
        ws.get(plan.ws_bytes)
        out = torch.empty(plan.out_shape, dtype=torch.float32, device=self.device)
        plan.forward(x, out, slot=0, training=training, ws=ws, drop_rate=drop_rate, drop_seed=drop_seed,
                     step_dev=self.arena.iterations)
        return out


class Discriminator(Network):
    """PatchGAN discriminator (pix2pix.py:194-220); called as D([inp, tar])."""
    kind = "pix2pix_discriminator"

    def __init__(self, width=1, seed=1235, device=None):
        super().__init__("discriminator", d_variables(width), d_layout_order(width), width, seed, device)

    def __call__(self, inputs, training=False):
        inp, tar = inputs
        inp, tar = to_device(inp, self.device), to_device(tar, self.device)
        N, H, W, _ = inp.shape
        plan = self._plan(("fwd", N, H, W),
                          lambda: DiscriminatorPlan(N, H, W, self.width, self.arena, self.bn, self.device, 1, False))
        ws = ops.Workspace(self.device)
        ws.get(plan.ws_bytes)
        ops.channel_concat(inp, tar, plan.slots[0]["inp"])
        plan.forward(slot=0, training=training, ws=ws)
        return plan.slots[0]["logits"].clone()


class Adam:
    """tf.keras.optimizers.Adam surface; TF ApplyAdam arithmetic on device.

    Moment slots live in the network's arena (same offsets as the variables),
    `iterations` is a device counter (read lazily; reading it synchronises)."""

    def __init__(self, learning_rate=1e-3, beta_1=0.9, beta_2=0.999, epsilon=1e-7, **kw):
        if "lr" in kw:
            learning_rate = kw.pop("lr")
        self.learning_rate, self.beta_1, self.beta_2, self.epsilon = learning_rate, beta_1, beta_2, epsilon
        self._arena = None

    lr = property(lambda self: self.learning_rate)

    def bind(self, arena):
        self._arena = arena
        return self

    @property
    def iterations(self):
        return int(self._arena.iterations.item()) if self._arena is not None else 0

    def current_lr(self):
        lr = self.learning_rate
        if callable(lr):
            return float(lr(self.iterations))
        return float(lr)

    def apply_gradients(self, grads_and_vars):
        """Per-variable update; every variable must be a view of the bound arena."""
        A = self._arena
        if A is None:
            raise ops.DGError("optimizer is not bound to a network (Pix2Pix binds it)")
        pairs = list(grads_and_vars)
        base = A.data.data_ptr()
        for g, v in pairs:
            off = (v.data_ptr() - base) // 4
            n = v.numel()
            if not (0 <= off and off + n <= A.numel):
                raise ops.DGError("variable is not part of this optimizer's network")
            g = g.contiguous()
            ops.adam(A.data[off:off + n], g.reshape(-1), A.m[off:off + n], A.v[off:off + n], self.current_lr(),
                     self.beta_1, self.beta_2, self.epsilon, A.iterations)
        ops.counter_add(A.iterations, 1)
