"""Sub-network containers of PhysicsNet, mirroring nn/network/blocks.py of the
reference module-for-module: same class names, same parameter names, shapes
and CREATION ORDER (so ``torch.manual_seed`` gives the reference's initial
weights and reference checkpoints load unchanged).

The training path runs them fused (``paig_reproduction_amd.engine``: the
whole PhysicsNet step at once).  Called one at a time, as the reference's
callers do, each forward below runs on the same HIP kernels through
``native_modules`` (differentiable; parameter gradients land in the owning
PhysicsNet's flat gradient buffer).
"""
import numpy as np
import torch.nn as pnn

from paig_reproduction_amd.nn.network import native_modules as _nm


class _ParamsOnly(pnn.Module):
    pass


class VelocityEncoder(_ParamsOnly):
    """nn/network/blocks.py:8-29 (MLP in*2 -> 100 -> 100 -> 2 with tanh, or the
    alt_vel linear map of position differences)."""

    def __init__(self, alt_vel, input_steps, n_objs, coord_units, device):
        super().__init__()
        self.alt_vel = alt_vel
        self.input_steps = input_steps
        self.n_objs = n_objs
        self.coord_units = coord_units
        self.device = device
        if self.alt_vel:
            self.init_vel_linear = pnn.Linear((self.input_steps - 1) * 2, 2)
        else:
            self.init_vel_mlp = pnn.Sequential(
                pnn.Linear(self.input_steps * self.coord_units // self.n_objs // 2, 100),
                pnn.Tanh(),
                pnn.Linear(100, 100),
                pnn.Tanh(),
                pnn.Linear(100, self.coord_units // self.n_objs // 2),
            )

    def forward(self, inp):
        """blocks.py:31-49: inp [B, input_steps, coord_units/2] -> [B, coord_units/2]."""
        return _nm.velocity_forward(self, inp)


class UNet(_ParamsOnly):
    """nn/network/blocks.py:106-170 (upsamp=True; Resize modules carry no params)."""

    def __init__(self, in_features, hidden_dim, out_features, upsamp=True):
        in_channels, height, width = in_features
        super().__init__()
        self.upsamp = upsamp
        hd = hidden_dim
        C = pnn.Conv2d
        self.c1 = C(in_channels, hd, kernel_size=3, padding="same")
        self.c2 = C(hd, hd, kernel_size=3, padding="same")
        self.c3 = C(hd, hd * 2, kernel_size=3, padding="same")
        self.c4 = C(hd * 2, hd * 2, kernel_size=3, padding="same")
        self.c5 = C(hd * 2, hd * 4, kernel_size=3, padding="same")
        self.c6 = C(hd * 4, hd * 4, kernel_size=3, padding="same")
        self.c7 = C(hd * 4, hd * 8, kernel_size=3, padding="same")
        if upsamp:
            self.c8 = C(hd * 8, hd * 8, kernel_size=3, padding="same")
        self.c9 = C(hd * 8, hd * 2, kernel_size=3, padding="same")
        self.c10 = C(hd * 6, hd * 4, kernel_size=3, padding="same")
        self.c11 = C(hd * 4, hd * 4, kernel_size=3, padding="same")
        if not upsamp:
            raise NotImplementedError("UNet(upsamp=False) is unused by the reference and not built")
        self.c12 = C(hd * 4, hd * 2, kernel_size=3, padding="same")
        self.c13 = C(hd * 4, hd * 2, kernel_size=3, padding="same")
        self.c14 = C(hd * 2, hd * 2, kernel_size=3, padding="same")
        self.c15 = C(hd * 2, hd * 2, kernel_size=3, padding="same")
        self.c16 = C(hd * 3, hd, kernel_size=3, padding="same")
        self.c17 = C(hd, hd, kernel_size=3, padding="same")
        self.c18 = C(hd, out_features, kernel_size=1, padding="same")

    def forward(self, x):
        """blocks.py:172-237: frames [N, 3, H, W] -> logits [N, n_objs, H, W] (c18 not ReLU'd)."""
        return _nm.unet_forward(self, x, "unet")


class ShallowUNet(_ParamsOnly):
    """nn/network/blocks.py:240-276."""

    def __init__(self, in_features, hidden_dim, out_features, upsamp=True):
        super().__init__()
        in_channels, height, width = in_features
        self.upsamp = upsamp
        if not upsamp:
            raise NotImplementedError("Using ShallowUNet without upsamp is not implemented yet")
        hd = hidden_dim
        C = pnn.Conv2d
        self.c1 = C(in_channels, hd, kernel_size=3, padding="same")
        self.c2 = C(hd, hd, kernel_size=3, padding="same")
        self.c3 = C(hd, hd * 2, kernel_size=3, padding="same")
        self.c4 = C(hd * 2, hd * 2, kernel_size=3, padding="same")
        self.c5 = C(hd * 2, hd * 4, kernel_size=3, padding="same")
        self.c6 = C(hd * 4, hd * 4, kernel_size=3, padding="same")
        self.c7 = C(hd * 4, hd * 2, kernel_size=3, padding="same")
        self.c8 = C(hd * 4, hd * 2, kernel_size=3, padding="same")
        self.c9 = C(hd * 2, hd * 2, kernel_size=3, padding="same")
        self.c10 = C(hd * 2, hd * 2, kernel_size=3, padding="same")
        self.c11 = C(hd * 3, hd, kernel_size=3, padding="same")
        self.c12 = C(hd, hd, kernel_size=3, padding="same")
        self.c13 = C(hd, out_features, kernel_size=1, padding="same")

    def forward(self, x):
        """blocks.py:278-308: frames [N, 3, H, W] -> ReLU'd logits [N, n_objs, H, W] (Q13)."""
        return _nm.unet_forward(self, x, "shallow_unet")


class ConvolutionalEncoder(_ParamsOnly):
    """nn/network/blocks.py:52-75: builds BOTH U-Nets (quirk Q8: the unused one
    stays in the state_dict and the RNG stream), then l1/l2/l3."""

    def __init__(self, in_features, hidden_dim, out_features, n_objects, device):
        super().__init__()
        self.device = device
        self.input_shape = in_features
        self.conv_ch = in_features[0]
        self.n_objs = n_objects
        self.shallow_unet = ShallowUNet(in_features, 8, n_objects, upsamp=True)
        self.unet = UNet(in_features, 16, n_objects)
        if self.input_shape[1] < 40:
            self.l1 = pnn.Linear(in_features[1] * in_features[1] * self.conv_ch, hidden_dim)
        else:
            self.l1 = pnn.Linear(in_features[1] // 2 * in_features[1] // 2 * self.conv_ch, hidden_dim)
        self.l2 = pnn.Linear(hidden_dim, hidden_dim)
        self.l3 = pnn.Linear(hidden_dim, out_features)

    def forward(self, inp):
        """blocks.py:77-103: frames [N, 3, H, W] -> (enc_pos [N, 2K] in pixels,
        enc_masks [N, K+1, H, W], masked_objs: K x [N, 3, H, W])."""
        return _nm.encoder_forward(self, inp)


class VariableFromNetwork(_ParamsOnly):
    """nn/network/blocks.py:311-316: l2(tanh(l1(ones[1,10]))) reshaped to `shape`."""

    def __init__(self, shape):
        super().__init__()
        self.l1 = pnn.Linear(10, 200)
        self.l2 = pnn.Linear(200, int(np.prod(shape)))
        self.shape = shape

    def forward(self):
        """blocks.py:318-322: l2(tanh(l1(ones[1, 10]))) reshaped to self.shape."""
        return _nm.vfn_forward(self)
