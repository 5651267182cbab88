"""keyBy exchange across the GPUs of one node: one process per GPU = one operator subtask.

Mirrors the reference's hash edge between source and window operator:
  routing   KeyGroupStreamPartitioner.selectChannels        SJ/runtime/partitioner/KeyGroupStreamPartitioner.java:52-65
            -> KeyGroupRangeAssignment.assignKeyToParallelOperator (kg * p / mp)  KeyGroupRangeAssignment.java:40-42,105-107
  transport RecordWriter.emit over local/remote channels    flink-runtime/.../io/network/api/writer/RecordWriter.java:82-85
  watermark RecordWriterOutput.emitWatermark -> broadcastEmit (RecordWriterOutput.java:80-84, RecordWriter.java:92-95);
            the receiver keeps one watermark per input channel, raised only when a larger one arrives, and
            forwards min over channels only when that minimum increases  SJ/runtime/io/StreamInputProcessor.java:147-161
MI355X form: the HIP partition kernel (fw_partition_by_operator_last) counting-sorts a batch by
destination in HBM with the rank's own share last; one all-to-all of per-destination counts, one MIN
all-reduce of the channels' watermarks, and the routed records: the other shares move as one group of
point-to-point sends/receives over xGMI (RCCL via torch.distributed backend "nccl": one group call for the
three columns of every peer), received into the same columns right behind the own share (a local channel:
never copied), and the whole goes to the engine in ONE push per step (a push carries a fixed device cost,
~15-20 us).

Every rank is both a source subtask (its own watermark = one input channel of every window subtask)
and a window subtask.  Because every watermark is broadcast, all window subtasks see the same channel
values: min over channels = MIN all-reduce of each source's monotone (max-so-far) watermark.

The GPU path is software-pipelined `depth` steps deep: step j enqueues the partition, the count
all-to-all and the watermark all-reduce of batch j and copies counts and watermark to pinned host memory
behind an event; the host then finishes batch j - depth (its counts arrived long ago): record
all-to-alls, the engine push and the watermark.  No host synchronisation waits on the batch just
enqueued.  `flush()` finishes the rest.  The same class runs on CPU tensors with the gloo backend for
the multi-process tests (routing by the numpy restatement in flink_amd.keygroups): either unpipelined
(`exchange()`), or through the very pipelined step()/_finish() code the GPUs run (`pipelined=True`: only
the partition kernel, the events and the device-side input waits are swapped for their host forms).

Skew: a rank may receive more records than its engine's max_batch (Zipf keys concentrate on a few key
groups); the received share is then pushed in max_batch pieces, all between the same two watermarks,
which is exact (a push is any run of records between watermarks, RecordWriter buffers any amount per
channel, RecordWriter.java:82-85).
"""
import ctypes
from collections import deque

import numpy as np
import torch
import torch.distributed as dist

from .keygroups import operator_index_np

LONG_MIN = -(1 << 63)


class _HostEvent:
    """The CPU path's stand-in for a torch.cuda.Event: host work is complete when it returns."""

    def record(self):
        pass

    def synchronize(self):
        pass


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
    # the engine records one consumption event per push in a ring of this many (fw_stream_wait_input)
    CONSUMED_RING = 8

    def __init__(self, engine, world, rank, max_parallelism, batch, device, depth=2, pipelined=None):
        self.eng = engine
        self.world, self.rank, self.mp = world, rank, max_parallelism
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.pipelined = self.cuda if pipelined is None else bool(pipelined)
        assert self.pipelined or not self.cuda, "the GPU path is pipelined"
        self.pushes = 0                 # engine pushes made (one per step; more only for a share above max_batch)
        self.local_wm = LONG_MIN        # this source's channel watermark, only raised
        self.last_emitted = LONG_MIN    # last watermark forwarded to the window subtask
        self.emitted = []               # the forwarded watermarks, in order (tests)
        if self.pipelined:
            if not 1 <= depth <= 3:
                # a send set returns every depth + 1 steps, each making up to two pushes: its last reader lies
                # at most 2 (depth + 1) - 1 pushes back, within the engine's ring of consumption events
                raise ValueError("KeyByExchange depth must be 1, 2 or 3")
            self.depth = depth
            S = self.depth + 1          # send sets: partition of batch j must not overwrite batch j - depth's
            z = lambda n, dt=torch.int64: torch.empty(n, dtype=dt, device=self.device)
            # a send set holds the batch sorted by destination with the own share last, then what the peers send
            # (received right behind it): batch + room for about a batch received; more (skew) regrows the set
            self.batch = batch
            cap = self._set_cap(batch)
            self.send = [(z(cap), z(cap), z(cap)) for _ in range(S)]
            # per send set: [send counts | received counts | aligned watermark] in one device tensor, read
            # back by one copy
            self.meta = [torch.zeros(2 * world + 1, dtype=torch.int64, device=self.device) for _ in range(S)]
            self.offsets = [torch.zeros(world, dtype=torch.int64, device=self.device) for _ in range(S)]
            host = (lambda x: x.pin_memory()) if self.cuda else (lambda x: x)
            self.host = [host(torch.zeros(2 * world + 1, dtype=torch.int64)) for _ in range(S)]
            self.local_wm_at = [LONG_MIN] * S   # world 1: the aligned watermark is the local one (host-known)
            self.ready = [torch.cuda.Event() if self.cuda else _HostEvent() for _ in range(S)]
            self.pending = deque()      # (set, batch size) staged, not yet finished
            self.staged = 0
            # engine push index that last read each send set: before a set is rewritten, torch's stream waits on
            # the device for the engine to have read it (fw_stream_wait_input), no host synchronisation
            self.send_pushed_at = [None] * S
            self.finished = self.pushes = 0
            # the engine enqueues its partition on torch's stream, so the exchange below is ordered after it
            if self.cuda:
                self.eng.use_stream(torch.cuda.current_stream(self.device).cuda_stream)

    # ------------------------------------------------------------------ routing
    @staticmethod
    def _set_cap(batch):
        return int(2.25 * batch) + 64

    def _dest_order(self):
        """Destinations in the order the partition writes them: the own share last."""
        return [(self.rank + 1 + i) % self.world for i in range(self.world)]

    def _route_cuda(self, k, t, v, si):
        n = k.numel()
        if n > self.batch:
            raise ValueError(f"batch of {n} records exceeds the exchange's batch capacity {self.batch}")
        P = lambda x: ctypes.c_void_p(x.data_ptr())
        sk, st, sv = self.send[si]
        rc = self.eng.lib.fw_partition_by_operator_last(self.eng.h, P(k), None, None, P(t), P(v), n, self.mp, self.world,
                                                        P(sk), None, None, P(st), P(sv), P(self.meta[si]),
                                                        P(self.offsets[si]), self.rank)
        if rc != 0:
            raise RuntimeError(f"fw_partition_by_operator_last failed: {rc}")

    def _route_into(self, k, t, v, si):
        """Partition a source batch into send set si (own share last) and its send counts (meta[si][:world])."""
        if self.cuda:
            self._route_cuda(k, t, v, si)
            return
        n = k.numel()
        if n > self.batch:
            raise ValueError(f"batch of {n} records exceeds the exchange's batch capacity {self.batch}")
        rk, rt, rv, counts = self._route_host(k, t, v, own_last=True)
        sk, st, sv = self.send[si]
        sk[:n].copy_(rk)
        st[:n].copy_(rt)
        sv[:n].copy_(rv.view(torch.int64) if rv.dtype == torch.float64 else rv)   # value bits, as the kernel writes
        self.meta[si][:self.world].copy_(counts)

    def _wait_read(self, pushed_at):
        """Before a send set or receive set is rewritten: the engine has read it (the push made at index
        pushed_at).  GPU: torch's stream waits on the device; beyond the event ring, or on CPU: a sync."""
        if pushed_at is None:
            return
        back = self.pushes - 1 - pushed_at
        if self.cuda and back < self.CONSUMED_RING:
            self.eng.wait_input(torch.cuda.current_stream(self.device).cuda_stream, back)
        else:
            self.eng.sync()

    def _push_share(self, cols3, count):
        """Push `count` records (one channel's share) to the engine in pieces of at most max_batch, all
        between the same two watermarks; returns the index of the last push that read them."""
        a, b, c = cols3
        as_value = (lambda x: x.view(torch.float64)) if self.eng.cfg.value_type == 1 else (lambda x: x)
        mb = int(self.eng.cfg.max_batch)
        for s0 in range(0, count, mb):
            s1 = min(count, s0 + mb)
            if self.cuda:
                self.eng.push(a[s0:s1], b[s0:s1], as_value(c[s0:s1]), keep_alive=False)
            else:
                self.eng.push(a[s0:s1].numpy(), b[s0:s1].numpy(), as_value(c[s0:s1]).numpy())
            self.pushes += 1
        return self.pushes - 1

    def _route_host(self, k, t, v, own_last=False):
        dest = operator_index_np(k.numpy(), self.mp, self.world)
        # stable by destination; with own_last in the partition kernel's order (the own share at the end)
        order = np.argsort((dest - self.rank - 1) % self.world if own_last else dest, kind="stable")
        counts = torch.from_numpy(np.bincount(dest, minlength=self.world).astype(np.int64))
        idx = torch.from_numpy(order)
        return k[idx], t[idx], v[idx], counts

    def _transfer(self, send, send_splits, recv_splits, recv, order=None):
        """The routed records between the ranks: `send` = (key, ts, value) sorted by destination (in `order`,
        default rank order) with send_splits per rank; the other ranks' shares land in `recv` (concatenated in
        rank order) through one group of point-to-point sends / receives.  Returns this rank's own share: views
        of `send` (a local channel, never copied).  Used by the GPU path (RCCL) and the CPU path (gloo) alike."""
        me, w = self.rank, self.world
        soff, o = [0] * (w + 1), 0
        for d in (order or range(w)):
            soff[d] = o
            o += send_splits[d]
        soff = {d: (soff[d], soff[d] + send_splits[d]) for d in range(w)}
        ops, roff = [], 0
        for p in range(w):
            if p == me:
                continue
            if recv_splits[p]:
                c = recv_splits[p]
                ops += [dist.P2POp(dist.irecv, x[roff:roff + c], p) for x in recv]
                roff += c
            if send_splits[p]:
                ops += [dist.P2POp(dist.isend, x[soff[p][0]:soff[p][1]], p) for x in send]
        if ops:
            for req in dist.batch_isend_irecv(ops):   # one group; on RCCL wait() orders torch's stream after it
                req.wait()
        return tuple(x[soff[me][0]:soff[me][1]] for x in send)

    def exchange(self, k, t, v):
        """CPU (gloo) path: route a source batch to the key-group owners; returns this rank's shares:
        [(key, ts, value) of its own records, (key, ts, value) received from the others]."""
        assert not self.cuda, "the GPU path is pipelined: use step() / flush()"
        sk, st, sv, counts = self._route_host(k, t, v)
        recv_counts = torch.empty_like(counts)
        dist.all_to_all_single(recv_counts, counts)
        send_splits, recv_splits = torch.stack([counts, recv_counts]).tolist()
        m = sum(recv_splits) - recv_splits[self.rank]
        recv = (torch.empty(m, dtype=torch.int64), torch.empty(m, dtype=torch.int64), torch.empty(m, dtype=v.dtype))
        own = self._transfer((sk, st, sv.contiguous()), send_splits, recv_splits, recv)
        return [own, recv]

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
        if not self.pipelined:
            # both shares between the same watermarks: one push, as the pipelined path
            own, recv = self.exchange(k, t, v)
            rk, rt, rv = (torch.cat([a, b]) for a, b in zip(own, recv))
            if rk.numel():
                self.eng.push(rk.numpy(), rt.numpy(), rv.numpy())
                self.pushes += 1
            self._forward(self.align_watermark(wm_local))
            return
        # finish the oldest batch first: its push then waits (device-side) for the partitions enqueued so far
        # only, and this batch's partition, enqueued below, overlaps with the engine's kernels of that batch
        while len(self.pending) >= self.depth:
            self._finish(*self.pending.popleft())
        si = self.staged % (self.depth + 1)
        self.staged += 1
        # the engine may still read this send set (the own share pushed from it): wait on the device
        self._wait_read(self.send_pushed_at[si])
        self._route_into(k, t, v, si)
        w, meta = self.world, self.meta[si]
        local = self._raise_local(wm_local)
        if w > 1:   # (one rank: its counts are its own receive counts, its watermark the aligned one)
            dist.all_to_all_single(meta[w:2 * w], meta[:w])
            meta[2 * w:].fill_(local)
            dist.all_reduce(meta[2 * w:], op=dist.ReduceOp.MIN)
        self.local_wm_at[si] = local
        self.host[si].copy_(meta, non_blocking=self.cuda)
        self.ready[si].record()
        self.pending.append((si, k.numel()))

    def flush(self):
        if self.pipelined:
            while self.pending:
                self._finish(*self.pending.popleft())

    def _finish(self, si, n):
        self.ready[si].synchronize()   # counts of a batch staged `depth` steps ago: normally long done
        h = self.host[si].tolist()
        w = self.world
        if w > 1:
            send_splits, recv_splits, aligned = h[:w], h[w:2 * w], h[2 * w]
        else:
            send_splits, recv_splits, aligned = h[:1], h[:1], self.local_wm_at[si]
        me = self.rank
        m = sum(recv_splits) - recv_splits[me]   # received from the other ranks
        own_n = send_splits[me]
        self.finished += 1
        sk, st, sv = self.send[si]
        if n + m > sk.numel():   # skew: more received than the set has room for behind the batch
            self.eng.sync()      # (nothing reads the old sets once the engine is idle)
            if self.cuda:        # (the partitions of the staged batches ran on this stream)
                torch.cuda.current_stream(self.device).synchronize()
            # every set grows to the new capacity at once: one engine sync per growth event, not one per
            # set as each meets the skew in turn; a set keeps the partitioned batch still staged in it
            cap = self._set_cap(n + m)
            staged = {sj: nj for sj, nj in self.pending}
            staged[si] = n
            for sj in range(len(self.send)):
                old = self.send[sj]
                if old[0].numel() >= cap:
                    continue
                grown = [torch.empty(cap, dtype=torch.int64, device=self.device) for _ in range(3)]
                keep = staged.get(sj, 0)
                for g, x in zip(grown, old):
                    g[:keep].copy_(x[:keep])
                self.send[sj] = tuple(grown)
            sk, st, sv = self.send[si]
        # the peers' shares land right behind the own share (the last destination of the partition's order)
        recv = (sk[n:n + m], st[n:n + m], sv[n:n + m])
        self._transfer((sk[:n], st[:n], sv[:n]), send_splits, recv_splits, recv, order=self._dest_order())
        # own share and received shares lie between the same watermarks: one push (a run above max_batch, under
        # skew, goes in pieces)
        if own_n + m:
            self.send_pushed_at[si] = self._push_share((sk[n - own_n:n + m], st[n - own_n:n + m], sv[n - own_n:n + m]),
                                                       own_n + m)
        self._forward(aligned)
