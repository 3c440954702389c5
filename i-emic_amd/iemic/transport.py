"""Host transport for the device library over torch.distributed (iemic_transport).

One process per subdomain, any device (several processes may share one GPU, where RCCL
refuses duplicate devices): the library stages its halo messages and sums in host memory
and calls these functions.  Pairing (include/iemic.h): the k-th message rank a sends to b
is the k-th b receives from a -- tagged here with per-peer counters on both sides.
"""
from __future__ import annotations

import collections
import ctypes as C

import numpy as np
import torch
import torch.distributed as dist

from . import _lib


class GlooTransport:
    """iemic_transport over an initialised torch.distributed process group (CPU tensors)."""

    def __init__(self, group=None):
        self.group = group
        self.ks = collections.Counter()
        self.kr = collections.Counter()
        self.pending = []
        self.c = _lib.Transport(None, _lib.SEND_FN(self._send), _lib.RECV_FN(self._recv),
                                _lib.WAIT_FN(self._wait), _lib.ALLRED_FN(self._allreduce))

    def _send(self, user, peer, buf, count):
        try:
            t = torch.from_numpy(np.ctypeslib.as_array(buf, shape=(count,)).copy())
            self.pending.append((dist.isend(t, peer, group=self.group, tag=self.ks[peer]), t))
            self.ks[peer] += 1
            return 0
        except Exception:
            return 1

    def _recv(self, user, peer, buf, count):
        try:
            t = torch.empty(count, dtype=torch.float64)
            dist.irecv(t, peer, group=self.group, tag=self.kr[peer]).wait()
            self.kr[peer] += 1
            np.ctypeslib.as_array(buf, shape=(count,))[:] = t.numpy()
            return 0
        except Exception:
            return 1

    def _wait(self, user):
        try:
            for req, _ in self.pending:
                req.wait()
            self.pending.clear()
            return 0
        except Exception:
            return 1

    def _allreduce(self, user, buf, count):
        try:
            a = np.ctypeslib.as_array(buf, shape=(count,))
            t = torch.from_numpy(a.copy())
            dist.all_reduce(t, group=self.group)
            a[:] = t.numpy()
            return 0
        except Exception:
            return 1
