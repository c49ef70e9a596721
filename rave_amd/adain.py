"""AdaIN buffers and the nn~ style-transfer controls of a model.

``AdaptiveInstanceNormalization`` (rave/blocks.py:856-919) keeps per-module
buffers mean_x, std_x, mean_y, std_y of shape (cc.MAX_BATCH_SIZE, C, 1) plus
the update counters num_update_x / num_update_y and the learn_x / learn_y
flags that nn~ exposes as the learn_source / learn_target attributes
(scripts/export.py:248-265).  The buffers live on the device inside the native
engine (include/rave_amd.h ``rave_model_adain_*``), where the AdaIN kernel
(rave_amd/csrc/adain.hip) reads and updates them in place; this class is the
host-side handle: flags, resets, and loading / reading the statistics under
the reference's state_dict names.

With no statistics loaded or learned (a fresh model) the module is the
identity and the offline plans contain no AdaIN op at all.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Mapping, Tuple

import numpy as np

from . import _native as N

MAX_BATCH_SIZE = 64   # cc.MAX_BATCH_SIZE, the buffers' leading dim (rave/blocks.py:860)
BUFFERS = ("mean_x", "std_x", "mean_y", "std_y")


class AdainState:
    """Buffers of every AdaIN module of a model, (name, channels) in graph order."""

    def __init__(self, model):
        self._m = model
        n = N.lib.rave_model_adain_count(model.handle)
        if n < 0:
            N.check(n, "adain_count")
        self.modules: List[Tuple[str, int]] = []
        name = C.create_string_buffer(256)
        ch, mb = C.c_int(), C.c_int()
        for i in range(n):
            N.check(N.lib.rave_model_adain_info(model.handle, i, name, 256, C.byref(ch), C.byref(mb)), "adain_info")
            self.modules.append((name.value.decode(), ch.value))
            self.max_batch = mb.value
        self.index: Dict[str, int] = {nm: i for i, (nm, _) in enumerate(self.modules)}
        self.learn_x = False
        self.learn_y = False
        self._touched = False

    @property
    def mode(self) -> int:
        """Kernel mode: 2 learn_y (checked first, as forward does), 1 learn_x, 0 transfer."""
        return 2 if self.learn_y else (1 if self.learn_x else 0)

    @property
    def active(self) -> bool:
        return self._touched or self.learn_x or self.learn_y

    # ------------------------------------------------------------ controls
    def _st(self):
        """The model device's current stream: resets queue behind the work on it."""
        import torch
        return C.c_void_p(torch.cuda.current_stream(self._m.device).cuda_stream)

    def set_learn(self, learn_x: bool = None, learn_y: bool = None) -> None:
        if learn_x is not None:
            self.learn_x = bool(learn_x)
        if learn_y is not None:
            self.learn_y = bool(learn_y)
        if self.learn_x or self.learn_y:
            self._touched = True
        N.check(N.lib.rave_model_adain_control(self._m.handle, -1 if learn_x is None else int(bool(learn_x)),
                                               -1 if learn_y is None else int(bool(learn_y)), 0, 0, self._st()), "adain")

    def reset_x(self) -> None:
        """AdaptiveInstanceNormalization.reset_x (rave/blocks.py:876-879)."""
        N.check(N.lib.rave_model_adain_control(self._m.handle, -1, -1, 1, 0, self._st()), "adain")

    def reset_y(self) -> None:
        """AdaptiveInstanceNormalization.reset_y (rave/blocks.py:881-884)."""
        N.check(N.lib.rave_model_adain_control(self._m.handle, -1, -1, 0, 1, self._st()), "adain")

    def _get(self, i: int) -> Tuple[np.ndarray, np.ndarray]:
        c = self.modules[i][1]
        st = np.empty((4, self.max_batch, c), np.float32)
        cnt = np.empty(2, np.float32)
        N.check(N.lib.rave_model_adain_get(self._m.handle, i, st.ctypes.data, cnt.ctypes.data), "adain_get")
        return st, cnt

    def load(self, state: Mapping[str, np.ndarray]) -> None:
        """Load the reference's buffers ``{module}.mean_x`` ... ``{module}.num_update_y``
        (state_dict names); missing entries keep their current values."""
        for i, (name, c) in enumerate(self.modules):
            st, cnt = self._get(i)
            hit = False
            for j, b in enumerate(BUFFERS):
                key = f"{name}.{b}"
                if key in state:
                    arr = np.asarray(state[key], np.float32).reshape(-1, c)
                    if arr.shape[0] > self.max_batch:
                        raise ValueError(f"{key}: {arr.shape[0]} rows > MAX_BATCH_SIZE {self.max_batch}")
                    st[j, :arr.shape[0]] = arr
                    hit = True
            for j, b in enumerate(("num_update_x", "num_update_y")):
                key = f"{name}.{b}"
                if key in state:
                    cnt[j] = float(np.asarray(state[key]).reshape(-1)[0])
                    hit = True
            if hit:
                N.check(N.lib.rave_model_adain_set(self._m.handle, i, st.ctypes.data, cnt.ctypes.data), "adain_set")
                self._touched = True

    def state_dict(self) -> Dict[str, np.ndarray]:
        """The buffers under the reference's names (shapes (MAX_BATCH, C, 1) and (1,))."""
        out: Dict[str, np.ndarray] = {}
        for i, (name, c) in enumerate(self.modules):
            st, cnt = self._get(i)
            for j, b in enumerate(BUFFERS):
                out[f"{name}.{b}"] = st[j][:, :, None].copy()
            out[f"{name}.num_update_x"] = cnt[0:1].copy()
            out[f"{name}.num_update_y"] = cnt[1:2].copy()
        return out
