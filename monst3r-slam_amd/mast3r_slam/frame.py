"""mast3r_slam.frame (frame.py:14-345) for one process: Frame / create_frame, the keyframe
store, the main loop's shared state and the per-frame pose log.  The reference shares
these between its frontend, backend and viewer processes through torch.multiprocessing and
a Manager; here they live in one process on the device (multi-process IPC is out of scope,
DESIGN.md §7), with the same methods the loop calls."""
from __future__ import annotations

import threading
from enum import Enum

import torch

from monst3r_slam_amd.global_opt import Keyframes
from monst3r_slam_amd.lie import Sim3
from monst3r_slam_amd.monst3r_utils import Frame, create_frame  # noqa: F401


class Mode(Enum):
    INIT = 0
    TRACKING = 1
    RELOC = 2
    TERMINATED = 3


class SharedKeyframes(Keyframes):
    """frame.py:243-345 (SharedKeyframes) over the device keyframe slabs."""

    def __init__(self, manager=None, h=384, w=512, buffer=512, dtype=torch.float32,
                 device="cuda"):
        super().__init__(h, w, buffer=buffer, device=device)
        self.lock = threading.RLock()

    def last_keyframe(self):
        with self.lock:
            return self[self.n_size - 1] if self.n_size else None

    def pop_last(self):
        with self.lock:
            self.n_size = max(0, self.n_size - 1)

    def set_intrinsics(self, K):
        self.K[:] = K

    def get_intrinsics(self):
        return self.K


class SharedStates:
    """frame.py: SharedStates — mode, the current frame, the backend task queues."""

    def __init__(self, manager=None, h=384, w=512, dtype=torch.float32, device="cuda"):
        self.lock = threading.RLock()
        self.mode = Mode.INIT
        self.paused = False
        self.global_optimizer_tasks = []
        self.edges_ii, self.edges_jj = [], []
        self.reloc_sem = _Counter()
        self._frame = None

    def set_mode(self, mode):
        with self.lock:
            self.mode = mode

    def get_mode(self):
        with self.lock:
            return self.mode

    def pause(self):
        self.paused = True

    def unpause(self):
        self.paused = False

    def is_paused(self):
        return self.paused

    def set_frame(self, frame):
        with self.lock:
            self._frame = frame

    def get_frame(self):
        with self.lock:
            return self._frame

    def queue_global_optimization(self, idx):
        with self.lock:
            self.global_optimizer_tasks.append(idx)

    def queue_reloc(self):
        with self.lock:
            self.reloc_sem.value += 1

    def dequeue_reloc(self):
        with self.lock:
            self.reloc_sem.value = max(0, self.reloc_sem.value - 1)


class _Counter:
    def __init__(self):
        self.value = 0


class SharedFramePoses:
    """frame.py: SharedFramePoses — every frame's (id, timestamp, T_WC) for
    save_full_traj."""

    def __init__(self, manager=None):
        self.frame_ids, self.timestamps, self.poses = [], [], []

    def add_pose(self, i, timestamp, T_WC):
        d = T_WC.data if isinstance(T_WC, Sim3) else T_WC
        self.frame_ids.append(int(i))
        self.timestamps.append(timestamp)
        self.poses.append(d.reshape(-1)[:8].detach().clone())

