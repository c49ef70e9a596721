"""Device-resident AdaIN buffers and the nn~ style-transfer controls.

``AdaptiveInstanceNormalization`` (rave/blocks.py:856-919) keeps per-module
buffers mean_x, std_x, mean_y, std_y of shape (cc.MAX_BATCH_SIZE, C, 1) plus
the update counters num_update_x / num_update_y and the learn_x / learn_y
flags that nn~ exposes as the learn_source / learn_target attributes.  Here
every module's buffers live in one device tensor that the AdaIN kernel reads
and updates in place (rave_amd/csrc/adain.hip); the learn flags are host-side
and select which kernel mode the recorded plans use.

With no learned statistics and no learning (a fresh model) the module is the
identity and the plans contain no AdaIN op at all.
"""
from __future__ import annotations

from typing import Dict, List, Mapping, Tuple

import numpy as np
import torch

MAX_BATCH_SIZE = 64   # cc.MAX_BATCH_SIZE, the buffers' leading dim (rave/blocks.py:860)
BUFFERS = ("mean_x", "std_x", "mean_y", "std_y")


class AdainState:
    """Buffers of every AdaIN module of a model, (name, channels) in graph order."""

    def __init__(self, modules: List[Tuple[str, int]], device, max_batch: int = MAX_BATCH_SIZE):
        self.modules = list(modules)
        self.max_batch = max_batch
        self.index: Dict[str, int] = {}
        self.offset: Dict[str, int] = {}
        off = 0
        for i, (name, c) in enumerate(self.modules):
            self.index[name] = i
            self.offset[name] = off
            off += 4 * max_batch * c
        self.stats = torch.empty(max(off, 1), dtype=torch.float32, device=device)
        self.counters = torch.zeros(max(len(self.modules), 1), 2, dtype=torch.float32, device=device)
        self.tickets = torch.zeros(max(len(self.modules), 1), dtype=torch.int32, device=device)
        self.learn_x = False
        self.learn_y = False
        self._touched = False          # any statistics loaded or learned
        self.reset_x()
        self.reset_y()
        self._touched = False

    # ------------------------------------------------------------ views
    def _view(self, name: str) -> torch.Tensor:
        c = self.modules[self.index[name]][1]
        o = self.offset[name]
        return self.stats[o:o + 4 * self.max_batch * c].view(4, self.max_batch, c)

    @property
    def mode(self) -> int:
        """Kernel mode: 2 learn_y (checked first, as forward does), 1 learn_x, 0 transfer."""
        return 2 if self.learn_y else (1 if self.learn_x else 0)

    @property
    def active(self) -> bool:
        return self._touched or self.learn_x or self.learn_y

    def key(self) -> tuple:
        return (self.active, self.mode)

    def ptrs(self, name: str) -> Tuple[int, int, int]:
        i = self.index[name]
        return (self.stats.data_ptr() + 4 * self.offset[name],
                self.counters.data_ptr() + 8 * i, self.tickets.data_ptr() + 4 * i)

    # ------------------------------------------------------------ controls
    def set_learn(self, learn_x: bool = None, learn_y: bool = None) -> None:
        if learn_x is not None:
            self.learn_x = bool(learn_x)
        if learn_y is not None:
            self.learn_y = bool(learn_y)
        if self.learn_x or self.learn_y:
            self._touched = True

    def reset_x(self) -> None:
        """AdaptiveInstanceNormalization.reset_x (rave/blocks.py:876-879)."""
        for name, _ in self.modules:
            v = self._view(name)
            v[0].zero_()
            v[1].fill_(1.0)
        self.counters[:, 0].zero_()

    def reset_y(self) -> None:
        """AdaptiveInstanceNormalization.reset_y (rave/blocks.py:881-884)."""
        for name, _ in self.modules:
            v = self._view(name)
            v[2].zero_()
            v[3].fill_(1.0)
        self.counters[:, 1].zero_()

    def load(self, state: Mapping[str, np.ndarray]) -> None:
        """Load the reference's buffers ``{module}.mean_x`` ... ``{module}.num_update_y``
        (state_dict names); missing entries keep their current values."""
        for name, c in self.modules:
            v = self._view(name)
            for j, b in enumerate(BUFFERS):
                key = f"{name}.{b}"
                if key in state:
                    arr = np.asarray(state[key], np.float32).reshape(-1, c)
                    if arr.shape[0] > self.max_batch:
                        raise ValueError(f"{key}: {arr.shape[0]} rows > MAX_BATCH_SIZE {self.max_batch}")
                    v[j, :arr.shape[0]].copy_(torch.from_numpy(arr))
                    self._touched = True
            for j, b in enumerate(("num_update_x", "num_update_y")):
                key = f"{name}.{b}"
                if key in state:
                    self.counters[self.index[name], j] = float(np.asarray(state[key]).reshape(-1)[0])
                    self._touched = True

    def state_dict(self) -> Dict[str, np.ndarray]:
        """The buffers under the reference's names (shapes (MAX_BATCH, C, 1) and (1,))."""
        out: Dict[str, np.ndarray] = {}
        cnt = self.counters.cpu().numpy()
        for name, c in self.modules:
            v = self._view(name).cpu().numpy()
            for j, b in enumerate(BUFFERS):
                out[f"{name}.{b}"] = v[j][:, :, None].copy()
            out[f"{name}.num_update_x"] = cnt[self.index[name], 0:1].copy()
            out[f"{name}.num_update_y"] = cnt[self.index[name], 1:2].copy()
        return out
