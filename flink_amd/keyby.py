"""keyBy exchange across the GPUs of one node: one process per GPU = one operator subtask.

Mirrors the reference's hash edge between source and window operator:
  routing   KeyGroupStreamPartitioner.selectChannels        SJ/runtime/partitioner/KeyGroupStreamPartitioner.java:52-65
            -> KeyGroupRangeAssignment.assignKeyToParallelOperator (kg * p / mp)  KeyGroupRangeAssignment.java:40-42,105-107
  transport RecordWriter.emit over local/remote channels    flink-runtime/.../io/network/api/writer/RecordWriter.java:82-85
  watermark RecordWriterOutput.emitWatermark -> broadcastEmit (RecordWriterOutput.java:80-84, RecordWriter.java:92-95),
            receiver takes the min over channels             SJ/runtime/io/StreamInputProcessor.java:147-161
MI355X form: the HIP partition kernel (fw_partition_by_operator) counting-sorts a batch by destination
in HBM; one all-to-all of per-destination counts, one all-to-all of the packed (key, ts, value)
records over xGMI (RCCL: torch.distributed backend "nccl"), one MIN all-reduce of the watermark.
The same class runs on CPU tensors with the gloo backend for the multi-process tests; there the
routing is the numpy restatement in flink_amd.keygroups (the GPU path always uses the HIP kernel).
"""
import ctypes

import numpy as np
import torch
import torch.distributed as dist

from .keygroups import operator_index_np


class KeyByExchange:
    def __init__(self, engine, world, rank, max_parallelism, batch, device):
        self.eng = engine
        self.world, self.rank, self.mp = world, rank, max_parallelism
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        if self.cuda:
            z = lambda dt=torch.int64: torch.empty(batch, dtype=dt, device=self.device)
            self.s_key, self.s_ts, self.s_val = z(), z(), z()
            self.counts = torch.zeros(world, dtype=torch.int64, device=self.device)
            self.offsets = torch.zeros(world, dtype=torch.int64, device=self.device)
            self.recv_counts = torch.zeros(world, dtype=torch.int64, device=self.device)
            self.RING = 3
            self.ring = [None] * self.RING
            self.pushed_at = [None] * self.RING   # engine push index that last read each set
            self.steps = self.pushes = 0
            self.pending_slot = None
            # the engine enqueues its partition on torch's stream, so the exchange below is ordered after it
            self.eng.use_stream(torch.cuda.current_stream(self.device).cuda_stream)

    def _route_cuda(self, k, t, v):
        n = k.numel()
        P = lambda x: ctypes.c_void_p(x.data_ptr())
        rc = self.eng.lib.fw_partition_by_operator(self.eng.h, P(k), None, None, P(t), P(v), n, self.mp, self.world,
                                                   P(self.s_key), None, None, P(self.s_ts), P(self.s_val),
                                                   P(self.counts), P(self.offsets))
        if rc != 0:
            raise RuntimeError(f"fw_partition_by_operator failed: {rc}")
        return self.s_key[:n], self.s_ts[:n], self.s_val[:n], self.counts

    def _route_host(self, k, t, v):
        dest = operator_index_np(k.numpy(), self.mp, self.world)
        order = np.argsort(dest, kind="stable")
        counts = torch.from_numpy(np.bincount(dest, minlength=self.world).astype(np.int64))
        idx = torch.from_numpy(order)
        return k[idx], t[idx], v[idx], counts

    def exchange(self, k, t, v):
        """Route a source batch to the key-group owners; returns this rank's received (key, ts, value)."""
        sk, st, sv, counts = self._route_cuda(k, t, v) if self.cuda else self._route_host(k, t, v)
        recv_counts = self.recv_counts if self.cuda else torch.empty_like(counts)
        dist.all_to_all_single(recv_counts, counts)
        splits = torch.stack([counts, recv_counts]).tolist()   # the one host synchronisation of the exchange
        send_splits, recv_splits = splits
        m = sum(recv_splits)
        if not self.cuda:
            packed = torch.stack([sk, st, sv.view(torch.int64)], dim=1)
            out = torch.empty((m, 3), dtype=torch.int64)
            dist.all_to_all_single(out, packed, recv_splits, send_splits)
            return out[:, 0].contiguous(), out[:, 1].contiguous(), out[:, 2].contiguous().view(v.dtype)
        # one all-to-all per column straight into the engine's input columns (no packing or unpacking
        # copy), from a ring of RING column sets: before a set is rewritten, torch's stream waits on the
        # device for the engine to have read it (fw_stream_wait_input), no host synchronisation
        slot = self.steps % self.RING
        cols = self.ring[slot]
        if cols is None or cols[0].numel() < m:
            if cols is not None:
                self.eng.sync()   # growing: the old set is dropped only once nothing reads it
            cap = max(m, int(1.25 * k.numel()))
            cols = self.ring[slot] = [torch.empty(cap, dtype=torch.int64, device=self.device) for _ in range(3)]
        elif self.pushed_at[slot] is not None:
            back = self.pushes - 1 - self.pushed_at[slot]
            if back < 8:
                self.eng.wait_input(torch.cuda.current_stream(self.device).cuda_stream, back)
        self.steps += 1
        self.pending_slot = slot
        rk, rt, rv = (x[:m] for x in cols)
        for dst, src in ((rk, sk), (rt, st), (rv, sv.view(torch.int64))):
            dist.all_to_all_single(dst, src, recv_splits, send_splits)
        return rk, rt, rv.view(v.dtype)

    def align_watermark(self, wm_local):
        """Min over all input channels (StreamInputProcessor.java:147-161)."""
        x = torch.tensor([wm_local], dtype=torch.int64, device=self.device)
        dist.all_reduce(x, op=dist.ReduceOp.MIN)
        return int(x.item())

    def step(self, k, t, v, wm_local):
        rk, rt, rv = self.exchange(k, t, v)
        if rk.numel():
            self.eng.push(rk, rt, rv, keep_alive=False)   # the ring keeps the columns (see exchange)
            if self.cuda:
                self.pushed_at[self.pending_slot] = self.pushes
                self.pushes += 1
        self.eng.advance_watermark(self.align_watermark(wm_local))
