"""The ASMC controller on its own: ``UsvAsmc`` (gym_usv/control/usv_asmc.py:4-244) over the HIP library.

``UsvAsmc`` keeps the reference's single-controller API -- ``compute(action, position, velocity,
do_perturb) -> (position, velocity, infos)`` on NumPy 3-vectors, and the ``so_filter`` (7),
``last`` (9), ``aux_vars`` (3) and ``perturb_step`` attributes (:43-49).  The reference's own tests
(tests/test_usv_asmc.py:8-37) call ``compute(a, p, v)`` and unpack two results, which the reference's
own ``compute`` (four arguments, three results) does not accept either; tests/test_gpu_r4.py runs
them in the adapted form ``p, v, _ = compute(a, p, v, False)``, as SURVEY §4 states.  ``UsvAsmcBatch`` is the batched form: n
independent controllers stepped in place on device tensors by one ``usv_asmc_compute`` launch.

Precision: "f64" (default, the reference's float64 arithmetic, the same substep function as the
env step's f64 build) or "f32".  There is no CPU fallback: without the library or a GPU the
constructors raise ``UsvLibError``.  ``infos`` is the empty list per call: the reference fills it
with per-substep diagnostics (``psi_d``, ``tport``, ...) that nothing on the path reads.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib

# state row -> reference attribute slot (usv_asmc.py:43-49; so_filter = [psi_d_last, o'', o', o,
# o, o', o''] since the reference keeps o_last = o, o_dot_last = o', o_dot_dot_last = o'' :89-92)
_SO_ROWS = (0, 3, 2, 1, 1, 2, 3)
_LAST_ROWS = tuple(range(4, 13))
_AUX_ROWS = (13, 14, 15)


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class UsvAsmcBatch:
    """n independent ``UsvAsmc`` controllers on one GPU.

    ``state`` is the [16, n] device tensor (rows: psi_d_last, o, o', o'', eta_dot_last[3],
    upsilon_dot_last[3], e_u_last, Ka_dot_u_last, Ka_dot_psi_last, e_u_int, Ka_u, Ka_psi);
    ``perturb_step`` the [n] int32 device tensor.  ``compute`` updates position / velocity
    ([n, 3] device tensors of the batch's dtype) in place and returns them.
    """

    def __init__(self, n, precision="f64", device=0):
        if not torch.cuda.is_available():
            raise _lib.UsvLibError("UsvAsmcBatch needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.lib = _lib.load()
        self.n = int(n)
        self.precision = {"f32": _lib.F32, "f64": _lib.F64}[precision]
        self.dtype = torch.float32 if precision == "f32" else torch.float64
        self.device = torch.device("cuda", device)
        self.state = torch.zeros((_lib.ASMC_STATE, self.n), dtype=self.dtype, device=self.device)
        self.perturb_step = torch.zeros(self.n, dtype=torch.int32, device=self.device)
        self.integral_step = 0.01                                       # usv_asmc.py:47

    def reset(self):
        """A fresh ``UsvAsmc()`` per controller (zero state, perturb_step 0)."""
        self.state.zero_()
        self.perturb_step.zero_()

    def _dev(self, x, cols):
        t = torch.as_tensor(x, device=self.device)
        if t.dtype != self.dtype or not t.is_contiguous():
            t = t.to(self.dtype).contiguous()
        if t.shape != (self.n, cols):
            raise ValueError(f"expected [{self.n}, {cols}], got {tuple(t.shape)}")
        return t

    def compute(self, action, position, velocity, do_perturb=False, calls=1):
        """``calls`` x UsvAsmc.compute (usv_asmc.py:53-244) on every controller.  ``position`` and
        ``velocity`` are updated in place when they are contiguous device tensors of the batch's
        dtype (else copies are), and returned."""
        a = self._dev(action, 2)
        p = self._dev(position, 3)
        v = self._dev(velocity, 3)
        # the library launches on the current device: make it this batch's, with the
        # launch on that device's current stream
        with torch.cuda.device(self.device):
            rc = self.lib.usv_asmc_compute(self.precision, self.n, ctypes.c_void_p(a.data_ptr()),
                                           ctypes.c_void_p(p.data_ptr()), ctypes.c_void_p(v.data_ptr()),
                                           ctypes.c_void_p(self.state.data_ptr()),
                                           ctypes.c_void_p(self.perturb_step.data_ptr()), int(bool(do_perturb)),
                                           int(calls), _stream(self.device))
        _lib.check(rc, self.lib)
        return p, v


class UsvAsmc:
    """HIP-backed ``UsvAsmc`` (gym_usv/control/usv_asmc.py:4) with the reference's NumPy API."""

    def __init__(self, precision="f64", device=0):
        self._b = UsvAsmcBatch(1, precision=precision, device=device)
        self.integral_step = 0.01

    # -- the reference's state attributes (usv_asmc.py:43-49), read from / written to the device
    def _rows(self, rows):
        st = self._b.state[:, 0].detach().cpu().numpy().astype(np.float64)
        return st[list(rows)]

    def _set_rows(self, rows, vals):
        vals = np.asarray(vals, dtype=np.float64).reshape(len(rows))
        st = self._b.state[:, 0].detach().cpu().numpy().astype(np.float64)
        for r, x in zip(rows, vals):
            st[r] = x
        self._b.state[:, 0] = torch.from_numpy(st).to(self._b.dtype)

    @property
    def so_filter(self):
        return self._rows(_SO_ROWS)

    @so_filter.setter
    def so_filter(self, vals):
        vals = np.asarray(vals, dtype=np.float64).reshape(7)
        if not (vals[1] == vals[6] and vals[2] == vals[5] and vals[3] == vals[4]):
            raise ValueError("so_filter must hold o_last == o, o_dot_last == o_dot, o_dot_dot_last == o_dot_dot "
                             "(the reference keeps them equal after every substep, usv_asmc.py:89-92)")
        self._set_rows((0, 3, 2, 1), vals[:4])

    @property
    def last(self):
        return self._rows(_LAST_ROWS)

    @last.setter
    def last(self, vals):
        self._set_rows(_LAST_ROWS, vals)

    @property
    def aux_vars(self):
        return self._rows(_AUX_ROWS)

    @aux_vars.setter
    def aux_vars(self, vals):
        self._set_rows(_AUX_ROWS, vals)

    @property
    def perturb_step(self):
        return int(self._b.perturb_step[0].item())

    @perturb_step.setter
    def perturb_step(self, k):
        self._b.perturb_step[0] = int(k)

    def compute(self, action, position, velocity, do_perturb):
        """usv_asmc.py:53-244: ten substeps of 0.01 s; returns (position, velocity, infos)."""
        a = np.asarray(action, dtype=np.float64).reshape(1, 2)
        p = np.asarray(position, dtype=np.float64).reshape(1, 3)
        v = np.asarray(velocity, dtype=np.float64).reshape(1, 3)
        p2, v2 = self._b.compute(a, p, v, do_perturb)
        return (p2[0].cpu().numpy().astype(np.float64), v2[0].cpu().numpy().astype(np.float64), [])
