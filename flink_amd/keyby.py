"""keyBy exchange across the GPUs of one node: one process per GPU = one operator subtask.

Mirrors the reference's hash edge between source and window operator:
  routing   KeyGroupStreamPartitioner.selectChannels        SJ/runtime/partitioner/KeyGroupStreamPartitioner.java:52-65
            -> KeyGroupRangeAssignment.assignKeyToParallelOperator (kg * p / mp)  KeyGroupRangeAssignment.java:40-42,105-107
  transport RecordWriter.emit over local/remote channels    flink-runtime/.../io/network/api/writer/RecordWriter.java:82-85
  watermark RecordWriterOutput.emitWatermark -> broadcastEmit (RecordWriterOutput.java:80-84, RecordWriter.java:92-95);
            the receiver keeps one watermark per input channel, raised only when a larger one arrives, and
            forwards min over channels only when that minimum increases  SJ/runtime/io/StreamInputProcessor.java:147-161
MI355X form: the HIP partition kernel (fw_partition_by_operator) counting-sorts a batch by destination
in HBM; one all-to-all of per-destination counts, per-column all-to-alls of the routed records over
xGMI (RCCL: torch.distributed backend "nccl"), one MIN all-reduce of the channels' watermarks.

Every rank is both a source subtask (its own watermark = one input channel of every window subtask)
and a window subtask.  Because every watermark is broadcast, all window subtasks see the same channel
values: min over channels = MIN all-reduce of each source's monotone (max-so-far) watermark.

The GPU path is software-pipelined `depth` steps deep: step j enqueues the partition, the count
all-to-all and the watermark all-reduce of batch j and copies counts and watermark to pinned host memory
behind an event; the host then finishes batch j - depth (its counts arrived long ago): record
all-to-alls, the engine push and the watermark.  No host synchronisation waits on the batch just
enqueued.  `flush()` finishes the rest.  The same class runs on CPU tensors with the gloo backend for
the multi-process tests (routing by the numpy restatement in flink_amd.keygroups, no pipelining).
"""
import ctypes
from collections import deque

import numpy as np
import torch
import torch.distributed as dist

from .keygroups import operator_index_np

LONG_MIN = -(1 << 63)


class ChannelWatermarks:
    """StreamInputProcessor's watermark valve (StreamInputProcessor.java:147-161) for a receiver whose
    input channels are the world's sources: per-channel maxima, emit min over channels on increase."""

    def __init__(self, channels):
        self.wm = [LONG_MIN] * channels
        self.last_emitted = LONG_MIN

    def on_watermark(self, channel, wm):
        """Returns the watermark to forward, or None."""
        if wm > self.wm[channel]:
            self.wm[channel] = wm
            new_min = min(self.wm)
            if new_min > self.last_emitted:
                self.last_emitted = new_min
                return new_min
        return None


class KeyByExchange:
    def __init__(self, engine, world, rank, max_parallelism, batch, device, depth=2):
        self.eng = engine
        self.world, self.rank, self.mp = world, rank, max_parallelism
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.local_wm = LONG_MIN        # this source's channel watermark, only raised
        self.last_emitted = LONG_MIN    # last watermark forwarded to the window subtask
        self.emitted = []               # the forwarded watermarks, in order (tests)
        if self.cuda:
            self.depth = max(1, depth)
            S = self.depth + 1          # send sets: partition of batch j must not overwrite batch j - depth's
            z = lambda n, dt=torch.int64: torch.empty(n, dtype=dt, device=self.device)
            self.send = [(z(batch), z(batch), z(batch)) for _ in range(S)]
            self.counts = [torch.zeros(world, dtype=torch.int64, device=self.device) for _ in range(S)]
            self.offsets = [torch.zeros(world, dtype=torch.int64, device=self.device) for _ in range(S)]
            self.recv_counts = [torch.zeros(world, dtype=torch.int64, device=self.device) for _ in range(S)]
            self.wm_dev = [torch.zeros(1, dtype=torch.int64, device=self.device) for _ in range(S)]
            self.host = [torch.zeros(2 * world + 1, dtype=torch.int64).pin_memory() for _ in range(S)]
            self.ready = [torch.cuda.Event() for _ in range(S)]
            self.pending = deque()      # (set, batch size) staged, not yet finished
            self.staged = 0
            # receive column sets: before a set is rewritten, torch's stream waits on the device for the
            # engine to have read it (fw_stream_wait_input), no host synchronisation
            self.RING = 3
            self.ring = [None] * self.RING
            self.pushed_at = [None] * self.RING   # engine push index that last read each set
            self.finished = self.pushes = 0
            # the engine enqueues its partition on torch's stream, so the exchange below is ordered after it
            self.eng.use_stream(torch.cuda.current_stream(self.device).cuda_stream)

    # ------------------------------------------------------------------ routing
    def _route_cuda(self, k, t, v, si):
        n = k.numel()
        if n > self.send[si][0].numel():
            raise ValueError(f"batch of {n} records exceeds the exchange's batch capacity {self.send[si][0].numel()}")
        P = lambda x: ctypes.c_void_p(x.data_ptr())
        sk, st, sv = self.send[si]
        rc = self.eng.lib.fw_partition_by_operator(self.eng.h, P(k), None, None, P(t), P(v), n, self.mp, self.world,
                                                   P(sk), None, None, P(st), P(sv), P(self.counts[si]),
                                                   P(self.offsets[si]))
        if rc != 0:
            raise RuntimeError(f"fw_partition_by_operator failed: {rc}")

    def _route_host(self, k, t, v):
        dest = operator_index_np(k.numpy(), self.mp, self.world)
        order = np.argsort(dest, kind="stable")
        counts = torch.from_numpy(np.bincount(dest, minlength=self.world).astype(np.int64))
        idx = torch.from_numpy(order)
        return k[idx], t[idx], v[idx], counts

    def exchange(self, k, t, v):
        """CPU (gloo) path: route a source batch to the key-group owners; returns this rank's received
        (key, ts, value)."""
        assert not self.cuda, "the GPU path is pipelined: use step() / flush()"
        sk, st, sv, counts = self._route_host(k, t, v)
        recv_counts = torch.empty_like(counts)
        dist.all_to_all_single(recv_counts, counts)
        send_splits, recv_splits = torch.stack([counts, recv_counts]).tolist()
        m = sum(recv_splits)
        packed = torch.stack([sk, st, sv.view(torch.int64)], dim=1)
        out = torch.empty((m, 3), dtype=torch.int64)
        dist.all_to_all_single(out, packed, recv_splits, send_splits)
        return out[:, 0].contiguous(), out[:, 1].contiguous(), out[:, 2].contiguous().view(v.dtype)

    # ------------------------------------------------------------------ watermarks
    def _raise_local(self, wm_local):
        self.local_wm = max(self.local_wm, int(wm_local))   # watermarks[channel] only increases
        return self.local_wm

    def align_watermark(self, wm_local):
        """Min over all input channels of each channel's max-so-far watermark (StreamInputProcessor.java:147-161)."""
        x = torch.tensor([self._raise_local(wm_local)], dtype=torch.int64, device=self.device)
        dist.all_reduce(x, op=dist.ReduceOp.MIN)
        return int(x.item())

    def _forward(self, aligned):
        """Forward the aligned watermark to the window subtask only if it increased."""
        if aligned > self.last_emitted:
            self.last_emitted = aligned
            self.emitted.append(aligned)
            self.eng.advance_watermark(aligned)

    # ------------------------------------------------------------------ one step
    def step(self, k, t, v, wm_local):
        """Source batch (k, t, v) followed by this source's watermark wm_local."""
        if not self.cuda:
            rk, rt, rv = self.exchange(k, t, v)
            if rk.numel():
                self.eng.push(rk.numpy(), rt.numpy(), rv.numpy())
            self._forward(self.align_watermark(wm_local))
            return
        si = self.staged % (self.depth + 1)
        self.staged += 1
        self._route_cuda(k, t, v, si)
        dist.all_to_all_single(self.recv_counts[si], self.counts[si])
        self.wm_dev[si].fill_(self._raise_local(wm_local))
        dist.all_reduce(self.wm_dev[si], op=dist.ReduceOp.MIN)
        h = self.host[si]
        w = self.world
        h[:w].copy_(self.counts[si], non_blocking=True)
        h[w:2 * w].copy_(self.recv_counts[si], non_blocking=True)
        h[2 * w:].copy_(self.wm_dev[si], non_blocking=True)
        self.ready[si].record()
        self.pending.append((si, k.numel()))
        while len(self.pending) > self.depth:
            self._finish(*self.pending.popleft())

    def flush(self):
        if self.cuda:
            while self.pending:
                self._finish(*self.pending.popleft())

    def _finish(self, si, n):
        self.ready[si].synchronize()   # counts of a batch staged `depth` steps ago: normally long done
        h = self.host[si].tolist()
        w = self.world
        send_splits, recv_splits, aligned = h[:w], h[w:2 * w], h[2 * w]
        m = sum(recv_splits)
        slot = self.finished % self.RING
        self.finished += 1
        cols = self.ring[slot]
        if cols is None or cols[0].numel() < m:
            if cols is not None:
                self.eng.sync()   # growing: the old set is dropped only once nothing reads it
            cap = max(m, int(1.25 * n))
            cols = self.ring[slot] = [torch.empty(cap, dtype=torch.int64, device=self.device) for _ in range(3)]
        elif self.pushed_at[slot] is not None:
            back = self.pushes - 1 - self.pushed_at[slot]
            if back < 8:
                self.eng.wait_input(torch.cuda.current_stream(self.device).cuda_stream, back)
        rk, rt, rv = (x[:m] for x in cols)
        sk, st, sv = self.send[si]
        for dst, src in ((rk, sk), (rt, st), (rv, sv)):
            dist.all_to_all_single(dst, src[:n], recv_splits, send_splits)
        if m:
            if m > self.eng.cfg.max_batch:
                raise ValueError(f"received {m} records, above the engine's max_batch {self.eng.cfg.max_batch}: "
                                 "size max_batch for the most skewed key-group range")
            self.eng.push(rk, rt, rv.view(torch.float64) if self.eng.cfg.value_type == 1 else rv, keep_alive=False)
            self.pushed_at[slot] = self.pushes
            self.pushes += 1
        self._forward(aligned)
