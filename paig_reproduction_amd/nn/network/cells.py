"""Physics cells, mirroring nn/network/cells.py of the reference: same
classes, the same RNNCell base (its unused weight_ih/weight_hh/bias_* stay in
the state_dict and the init RNG stream, quirk Q8) and the same parameters
(dt fp32 frozen; k, equil / g, m 0-dim fp64, quirk Q9).

The integrators themselves run fused over all rollout steps in the HIP kernel
``paig_rollout_fwd/bwd`` (csrc/rollout.hip), which restates
spring (:31-51), bouncing (:60-83) and gravity (:96-106) exactly, including
the split-size-1 quirk Q3.  Gravity recomputes A = exp(g) exp(2m) per step
(the reference computes it once in __init__, Q4)."""
import numpy as np
import torch
import torch.nn as tnn


class ode_cell(tnn.RNNCell):
    def __init__(self, input_size, hidden_size):
        super().__init__(input_size, hidden_size)
        self.input_size = input_size
        self.hidden_size = hidden_size

    @property
    def state_size(self):
        return self.hidden_size, self.hidden_size

    def zero_state(self, batch_size, dtype):
        x_0 = torch.zeros(batch_size, self.hidden_size, dtype=dtype)
        v_0 = torch.zeros(batch_size, self.hidden_size, dtype=dtype)
        return x_0, v_0

    def forward(self, poss, vels):
        """One cell step (5 substeps) on paig_rollout_fwd/bwd with R = 1:
        poss, vels [B, coord_units/2] -> (poss, vels).  The training path runs
        all R steps in one launch instead (PhysicsNet.forward)."""
        from paig_reproduction_amd.nn.network import native_modules as _nm
        return _nm.cell_forward(self, poss, vels)


class spring_ode_cell(ode_cell):
    """ Assumes there are 2 objects """
    KIND = 0

    def __init__(self, input_size, hidden_size):
        super().__init__(input_size, hidden_size)
        self.dt = tnn.Parameter(torch.tensor(0.3), requires_grad=False)
        self.k = tnn.Parameter(torch.tensor(np.log(1.0)), requires_grad=True)
        self.equil = tnn.Parameter(torch.tensor(np.log(1.0)), requires_grad=True)


class bouncing_ode_cell(ode_cell):
    """ Assumes there are 2 objects """
    KIND = 1

    def __init__(self, input_size, hidden_size):
        super().__init__(input_size, hidden_size)
        self.dt = tnn.Parameter(torch.tensor(0.3), requires_grad=False)


class gravity_ode_cell(ode_cell):
    """ Assumes there are 3 objects """
    KIND = 2

    def __init__(self, input_size, hidden_size):
        super().__init__(input_size, hidden_size)
        self.dt = tnn.Parameter(torch.tensor(0.5), requires_grad=False)
        self.g = tnn.Parameter(torch.tensor(np.log(1.0)), requires_grad=True)
        self.m = tnn.Parameter(torch.tensor(np.log(1.0)), requires_grad=False)

    @property
    def A(self):
        return torch.exp(self.g.detach()) * torch.exp(2 * self.m.detach())
