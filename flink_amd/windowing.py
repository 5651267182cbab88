"""Host mirror of the reference's event-time window operator surface, driving the HIP engine.

Names and behaviour follow the reference (paths relative to the reference root,
SJ = flink-streaming-java/src/main/java/org/apache/flink/streaming/):
  TumblingEventTimeWindows.of(size[, offset])   SJ/api/windowing/assigners/TumblingEventTimeWindows.java:92-116
  SlidingEventTimeWindows.of(size, slide[, off]) SJ/api/windowing/assigners/SlidingEventTimeWindows.java:107-133
  EventTimeTrigger.create()                      SJ/api/windowing/triggers/EventTimeTrigger.java
  PurgingTrigger.of(trigger)                     SJ/api/windowing/triggers/PurgingTrigger.java
  WindowOperator.processElement/processWatermark SJ/runtime/operators/windowing/WindowOperator.java:222-375
  StreamRecord / Watermark                       SJ/runtime/streamrecord/StreamRecord.java, SJ/api/watermark/Watermark.java

The Java operator hands the engine one batch per watermark epoch (all records between two
watermarks see the same current watermark, StreamInputProcessor.java:147-177), so batching
records until the next watermark is exactly equivalent to per-record processing.
"""
import ctypes

import numpy as np

from . import _abi
from .keygroups import DEFAULT_MAX_PARALLELISM

LONG_MIN = -(1 << 63)
LONG_MAX = (1 << 63) - 1


def _java_rem(a, b):
    """Java `%` on longs (truncating toward zero)."""
    r = abs(a) % abs(b)
    return -r if a < 0 else r


def java_string_hash(s):
    h = 0
    for ch in s:
        h = (31 * h + ord(ch)) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


# ------------------------------------------------------------------ assigners / triggers
class TumblingEventTimeWindows:
    def __init__(self, size, offset):
        self.size, self.offset, self.slide = size, offset, size

    @staticmethod
    def of(size, offset=None):
        if offset is None:
            return TumblingEventTimeWindows(size, 0)
        return TumblingEventTimeWindows(size, _java_rem(offset, size))

    kind = _abi.FW_TUMBLING


class SlidingEventTimeWindows:
    def __init__(self, size, slide, offset):
        self.size, self.slide, self.offset = size, slide, offset

    @staticmethod
    def of(size, slide, offset=None):
        if offset is None:
            return SlidingEventTimeWindows(size, slide, 0)
        return SlidingEventTimeWindows(size, slide, _java_rem(offset, slide))

    kind = _abi.FW_SLIDING


class EventTimeSessionWindows:
    """EventTimeSessionWindows.withGap(gap) (SJ/api/windowing/assigners/EventTimeSessionWindows.java:53-56,
    :75-77): each record opens [ts, ts + gap); windows that intersect merge (TimeWindow.mergeWindows
    :186-230), the merging branch of WindowOperator (:228-301) keeps them per key."""

    def __init__(self, gap):
        self.size, self.slide, self.offset = gap, 0, 0

    @staticmethod
    def withGap(gap):
        return EventTimeSessionWindows(gap)

    kind = _abi.FW_SESSION


class EventTimeTrigger:
    code = _abi.FW_TRIGGER_EVENT_TIME

    @staticmethod
    def create():
        return EventTimeTrigger()


class PurgingTrigger:
    code = _abi.FW_TRIGGER_PURGING_EVENT_TIME

    def __init__(self, nested):
        if not isinstance(nested, EventTimeTrigger):
            raise NotImplementedError("only PurgingTrigger.of(EventTimeTrigger.create()) is on the GPU path")
        self.nested = nested

    @staticmethod
    def of(nested):
        return PurgingTrigger(nested)


class ReduceFunction:
    """The reduce functions the engine implements, as (record -> accumulator) field sets.

    A record is (key, f1, value).  reduce(value1 = stored, value2 = new) returns value1 with
    sum = v1 + v2, min = Math.min, max = Math.max, count = c1 + c2; f1 stays value1's (first arrival).
    comparable=True orders min/max by Double.compareTo instead (ComparableAggregator .min/.max).
    "maxBy" / "minBy" return the extremal record itself, value and f1 (ComparableAggregator MAXBY/MINBY,
    ComparableAggregator.java:74-81), a tie keeping the earlier record when first=True.
    `SumReducer()` is WindowOperatorTest.SumReducer (WindowOperatorTest.java:2245-2252).
    """
    FIELDS = {"sum": _abi.FW_AGG_SUM, "min": _abi.FW_AGG_MIN, "max": _abi.FW_AGG_MAX, "count": _abi.FW_AGG_COUNT,
              "maxBy": _abi.FW_AGG_MAXBY, "minBy": _abi.FW_AGG_MINBY}
    COLUMN = {"sum": "sum", "min": "min", "max": "max", "count": "count", "maxBy": "max", "minBy": "min"}

    def __init__(self, fields=("sum",), value_type="i64", keep_first_f1=False, comparable=False, first=True):
        self.fields = tuple(fields)
        self.mask = 0
        for f in self.fields:
            self.mask |= self.FIELDS[f]
        self.by = bool(self.mask & (_abi.FW_AGG_MAXBY | _abi.FW_AGG_MINBY))
        if self.by and len(self.fields) != 1:
            raise ValueError("maxBy / minBy return the whole record and combine with no other field")
        self.value_type = value_type
        self.keep_first_f1 = keep_first_f1 or self.by   # maxBy/minBy: the extremal record's f1
        self.comparable = comparable
        self.first = first
        self.flags = (_abi.FW_AGGF_COMPARABLE if comparable else 0) | (0 if first else _abi.FW_AGGF_BY_LAST)

    @property
    def vt(self):
        return _abi.FW_VALUE_I64 if self.value_type == "i64" else _abi.FW_VALUE_F64


class FoldFunction:
    """WindowedStream.fold(initialValue, foldFunction) (WindowedStream.java:213-242) for the folds the engine
    computes: "sum" (acc, v) -> acc + v, "count" (acc, v) -> acc + 1, "min" / "max" (acc, v) -> Math.min/max(acc, v),
    starting from `initial` (HeapFoldingState.add, HeapFoldingState.java:111-118: the first record folds into the
    descriptor's default value).  The result of a window is the accumulator."""
    KINDS = {"sum": _abi.FW_AGG_SUM, "count": _abi.FW_AGG_COUNT, "min": _abi.FW_AGG_MIN, "max": _abi.FW_AGG_MAX}

    def __init__(self, kind, initial, value_type="i64"):
        if kind not in self.KINDS:
            raise ValueError(f"fold {kind!r}: the GPU path folds sum, count, min or max")
        self.fields = (kind,)
        self.mask = self.KINDS[kind]
        self.value_type = value_type
        self.keep_first_f1 = False
        self.by = False
        self.comparable = False
        self.first = True
        self.flags = _abi.FW_AGGF_FOLD
        self.initial = initial
        if kind != "count" and value_type == "f64":   # a double accumulator: its bits
            self.initial_bits = int(np.array([float(initial)], np.float64).view(np.int64)[0])
        else:
            self.initial_bits = int(initial)

    @property
    def vt(self):
        return _abi.FW_VALUE_I64 if self.value_type == "i64" else _abi.FW_VALUE_F64


class ListStateDescriptor:
    """The window contents of WindowedStream.apply(WindowFunction) (WindowedStream.java:244-345): every element
    is kept (HeapListState, HeapListState.java:84-112) and the window function sees all of a key's elements of
    a firing window in arrival order (InternalIterableWindowFunction).  The engine buffers and groups them on
    the GPU; the window function runs on the host per (key, window) group.  `list_capacity`: elements buffered
    per pane slice (0: 4 x max_batch)."""

    def __init__(self, value_type="i64", list_capacity=0):
        self.fields = ()
        self.mask = _abi.FW_AGG_LIST
        self.value_type = value_type
        self.keep_first_f1 = True
        self.by = False
        self.comparable = False
        self.first = True
        self.flags = 0
        self.list_capacity = list_capacity

    @property
    def vt(self):
        return _abi.FW_VALUE_I64 if self.value_type == "i64" else _abi.FW_VALUE_F64


def SumReducer(value_type="i64"):
    return ReduceFunction(("sum",), value_type)


class Aggregations:
    """The built-in window aggregations of WindowedStream (WindowedStream.java:523-713) over the record's
    value field: sum (SumAggregator), min/max (ComparableAggregator MIN/MAX: value1's other fields, the
    field set to the extremum in compareTo order) and minBy/maxBy (the extremal record)."""

    @staticmethod
    def sum(value_type="i64"):
        return ReduceFunction(("sum",), value_type, keep_first_f1=True)

    @staticmethod
    def min(value_type="i64"):
        return ReduceFunction(("min",), value_type, keep_first_f1=True, comparable=True)

    @staticmethod
    def max(value_type="i64"):
        return ReduceFunction(("max",), value_type, keep_first_f1=True, comparable=True)

    @staticmethod
    def minBy(value_type="i64", first=True):
        return ReduceFunction(("minBy",), value_type, first=first)

    @staticmethod
    def maxBy(value_type="i64", first=True):
        return ReduceFunction(("maxBy",), value_type, first=first)


# ------------------------------------------------------------------ windows / window functions
class TimeWindow:
    """[start, end); maxTimestamp() = end - 1 (SJ/api/windowing/windows/TimeWindow.java:41-62)."""
    __slots__ = ("start", "end")

    def __init__(self, start, end):
        self.start, self.end = start, end

    def getStart(self):
        return self.start

    def getEnd(self):
        return self.end

    def maxTimestamp(self):
        return self.end - 1

    def __eq__(self, o):
        return isinstance(o, TimeWindow) and (self.start, self.end) == (o.start, o.end)

    def __hash__(self):
        return hash((self.start, self.end))

    def __repr__(self):
        return f"TimeWindow{{start={self.start}, end={self.end}}}"


class Collector:
    """org.apache.flink.util.Collector: what a WindowFunction emits."""

    def __init__(self):
        self.items = []

    def collect(self, record):
        self.items.append(record)


# ------------------------------------------------------------------ stream elements
class StreamRecord:
    __slots__ = ("value", "timestamp")

    def __init__(self, value, timestamp):
        self.value, self.timestamp = value, timestamp

    def __repr__(self):
        return f"StreamRecord({self.value!r}, {self.timestamp})"

    def __eq__(self, o):
        return isinstance(o, StreamRecord) and self.value == o.value and self.timestamp == o.timestamp

    def __hash__(self):
        return hash((self.value, self.timestamp))


class Watermark:
    __slots__ = ("timestamp",)

    def __init__(self, timestamp):
        self.timestamp = timestamp

    def __repr__(self):
        return f"Watermark({self.timestamp})"

    def __eq__(self, o):
        return isinstance(o, Watermark) and o.timestamp == self.timestamp

    def __hash__(self):
        return hash(("wm", self.timestamp))


# ------------------------------------------------------------------ engine wrapper
def _ptr(a):
    """Pointer of a numpy array or a torch tensor (device pointer for GPU tensors)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data_as(ctypes.c_void_p)
    return ctypes.c_void_p(a.data_ptr())


def _is_device(a):
    return a is not None and not isinstance(a, np.ndarray) and getattr(a, "is_cuda", False)


class WindowEngine:
    """One fw_engine (one operator subtask on one GPU) behind the C-ABI."""

    def __init__(self, config, lib=None, prefix="fw"):
        self.lib = lib if lib is not None else _abi.load_library()
        self.prefix = prefix
        self.cfg = config
        h = ctypes.c_void_p()
        rc = self._fn("create")(ctypes.byref(config), ctypes.byref(h))
        if rc != 0:
            raise _abi.FwError(rc, self._fn("last_error")(None).decode() or "fw_create failed")
        self.h = h
        self._inflight = []   # device columns pushed since the last sync/collect (read asynchronously)
        self._drain_keep = {}   # drain ticket -> inputs pushed before it (collect_begin / collect_end)

    def _fn(self, name):
        return getattr(self.lib, f"{self.prefix}_{name}")

    def _check(self, rc):
        if rc != 0:
            raise _abi.FwError(rc, self._fn("last_error")(self.h).decode())

    def use_stream(self, stream_handle):
        """Make an external HIP stream the producer of pushed columns (e.g. torch.cuda.current_stream().cuda_stream):
        each push waits for the work enqueued on it so far."""
        if self.prefix == "fw":
            self._check(self._fn("set_stream")(self.h, ctypes.c_void_p(stream_handle)))
            self._stream = stream_handle

    def wait_input(self, stream_handle, back):
        """Make an external HIP stream wait (on the device) until the engine has read the columns of the push
        made `back` non-empty pushes ago (fw_stream_wait_input)."""
        self._check(self._fn("stream_wait_input")(self.h, ctypes.c_void_p(stream_handle), back))

    def push(self, key, ts, value, key_hash=None, f1=None, keep_alive=True):
        n = len(key)
        if self.prefix == "fw":
            mem = _abi.FW_MEM_DEVICE if _is_device(key) else _abi.FW_MEM_HOST
            if mem == _abi.FW_MEM_DEVICE:
                # device columns are produced on torch's current stream: the engine waits for it at each
                # push, and reads the columns on its own streams until a later sync/collect, so the
                # tensors are kept alive until then (torch's allocator does not see the engine's streams)
                import torch
                cur = torch.cuda.current_stream(key.device).cuda_stream
                if getattr(self, "_stream", None) != cur:
                    self.use_stream(cur)
                if keep_alive:
                    self._inflight.append((key, ts, value, key_hash, f1))
            self._check(self._fn("push_batch")(self.h, _ptr(key), _ptr(key_hash), _ptr(f1), _ptr(ts), _ptr(value), n, mem))
        else:
            self._check(self._fn("push_batch")(self.h, _ptr(key), _ptr(key_hash), _ptr(f1), _ptr(ts), _ptr(value), n))

    def advance_watermark(self, wm):
        self._check(self._fn("advance_watermark")(self.h, wm))

    def sync(self):
        if self.prefix == "fw":
            self._check(self._fn("sync")(self.h))
            self._inflight.clear()
            self._drain_keep = {t: 0 for t in self._drain_keep}

    def collect_begin(self):
        """Start an asynchronous drain of the results since the last collect (fw_collect_begin): returns a ticket for
        collect_end; the batches pushed meanwhile run while the results travel to the host."""
        t = ctypes.c_int32()
        self._check(self._fn("collect_begin")(self.h, ctypes.byref(t)))
        self._drain_keep[t.value] = len(self._inflight)   # inputs pushed before the drain: read once it lands
        return t.value

    def collect_end(self, ticket, copy=True):
        """The drain `ticket` (collect_begin) once it has landed: the same dict as collect().  copy=False returns
        views of the pinned host columns instead (no copy; valid until the next collect_begin, as the C-ABI
        says), the way a JNI operator reads them."""
        o = _abi.FwOut()
        self._check(self._fn("collect_end")(self.h, ticket, ctypes.byref(o)))
        done = self._drain_keep.pop(ticket, 0)
        del self._inflight[:done]
        for t in self._drain_keep:
            self._drain_keep[t] = max(0, self._drain_keep[t] - done)
        return self._out_dict(o, copy)

    def collect(self):
        """Results since the last collect: dict of numpy columns + (mark_wm, mark_pos)."""
        o = _abi.FwOut()
        if self.prefix == "fw":
            self._check(self._fn("collect")(self.h, ctypes.byref(o), _abi.FW_MEM_HOST))
            self._inflight.clear()
            self._drain_keep = {t: 0 for t in self._drain_keep}
        else:
            self._check(self._fn("collect")(self.h, ctypes.byref(o)))
        return self._out_dict(o)

    def _out_dict(self, o, copy=True):
        n = o.n
        res = {"n": n}
        cp = (lambda a: a.copy()) if copy else (lambda a: a)
        for name in ("key", "f1", "ts", "sum_i64", "min_i64", "max_i64", "count", "sum_f64", "min_f64", "max_f64"):
            p = getattr(o, name)
            if n == 0:
                res[name] = np.zeros(0, np.float64 if name.endswith("f64") else np.int64)
            else:
                res[name] = cp(np.ctypeslib.as_array(p, shape=(n,))) if p else None
        nm = o.n_marks
        res["win_start"] = (cp(np.ctypeslib.as_array(o.win_start, shape=(n,))) if o.win_start
                            else (np.zeros(0, np.int64) if n == 0 else None))
        res["mark_wm"] = np.ctypeslib.as_array(o.mark_wm, shape=(nm,)).copy() if nm > 0 else np.zeros(0, np.int64)
        res["mark_pos"] = np.ctypeslib.as_array(o.mark_pos, shape=(nm,)).copy() if nm > 0 else np.zeros(0, np.int64)
        if self.prefix != "fw":
            self._fn("clear_output")(self.h)
        return res

    def snapshot_kg(self, kg):
        """State of key group kg as one blob (fw_snapshot_kg; HeapKeyedStateBackend.writeStateTableForKeyGroup
        + HeapInternalTimerService.snapshotTimersForKeyGroup)."""
        n = ctypes.c_int64()
        self._check(self._fn("snapshot_kg")(self.h, kg, None, 0, ctypes.byref(n)))
        buf = np.zeros(n.value // 8, dtype=np.int64)
        self._check(self._fn("snapshot_kg")(self.h, kg, _ptr(buf), n.value, ctypes.byref(n)))
        return buf.tobytes()

    def restore_kg(self, kg, blob):
        """Load a key group's blob before the first push (fw_restore_kg; readStateTableForKeyGroup)."""
        buf = np.frombuffer(blob, dtype=np.int64).copy()
        self._check(self._fn("restore_kg")(self.h, kg, _ptr(buf), len(blob)))

    def snapshot_kg_flink(self, kg, layout):
        """Key group kg in the reference's checkpoint layout (fw_snapshot_kg_flink): (state, timers) bytes —
        the managed keyed-state section at KeyGroupRangeOffsets[kg] (HeapKeyedStateBackend.java:196-248) and
        the body of HeapInternalTimerService.snapshotTimersForKeyGroup (:285-310).  `layout` names the state
        tuple's fields in order: "key", "f1", "sum", "min", "max", "count", "value" (maxBy/minBy)."""
        L = state_layout(layout)
        ns, nt = ctypes.c_int64(), ctypes.c_int64()
        fn = self._fn("snapshot_kg_flink")
        self._check(fn(self.h, kg, ctypes.byref(L), None, 0, ctypes.byref(ns), None, 0, ctypes.byref(nt)))
        st = ctypes.create_string_buffer(max(ns.value, 1))
        tm = ctypes.create_string_buffer(max(nt.value, 1))
        self._check(fn(self.h, kg, ctypes.byref(L), st, ns.value, ctypes.byref(ns), tm, nt.value, ctypes.byref(nt)))
        return st.raw[:ns.value], tm.raw[:nt.value]

    def restore_kg_flink(self, kg, layout, state, timers, watermark=-(1 << 63)):
        """Load a key group written in the reference's layout before the first push (fw_restore_kg_flink;
        readStateTableForKeyGroup + restoreTimersForKeyGroup).  The default watermark is the reference's:
        its timer service restarts at Long.MIN_VALUE."""
        L = state_layout(layout)
        sb = ctypes.create_string_buffer(bytes(state), max(len(state), 1))
        tb = ctypes.create_string_buffer(bytes(timers), max(len(timers), 1))
        self._check(self._fn("restore_kg_flink")(self.h, kg, ctypes.byref(L), watermark, sb, len(state), tb,
                                                 len(timers)))

    def decode(self, data, fields, key=0, value=None, f1=None, record_cap=None, marker_cap=1 << 16, device=False,
               buffers=None):
        """Decode Flink network-buffer bytes (fw_decode: length-prefixed StreamElementSerializer elements over a
        TupleSerializer tuple) into record columns, watermarks and latency markers in stream order.

        data: bytes / numpy uint8 (host) or a torch uint8 tensor on the GPU; fields: the tuple's field types
        ("long", "double", "int"); key / value / f1: field indices (f1 None: the record timestamp).  Returns a
        dict of numpy arrays (device=True: torch tensors on the engine's GPU, ready for push) and the counts;
        "consumed" < len(data) when the bytes end inside an element.  buffers: a previous result's "buffers" (the same
        capacities) to decode into again instead of allocating the output columns."""
        return self.decode_end(self.decode_begin(data, fields, key, value, f1, record_cap, marker_cap, device, buffers))

    def decode_begin(self, data, fields, key=0, value=None, f1=None, record_cap=None, marker_cap=1 << 16, device=False,
                     buffers=None):
        """fw_decode_begin: enqueue the decode and return a handle for decode_end (the same dict as decode()); the
        next buffer's decode can be enqueued before this one's counts are read back (two outstanding at most)."""
        types = {"long": _abi.FW_FT_LONG, "double": _abi.FW_FT_DOUBLE, "int": _abi.FW_FT_INT}
        sc = _abi.FwTupleSchema()
        sc.n_fields = len(fields)
        for i, f in enumerate(fields):
            sc.field_type[i] = types[f]
        sc.key_field, sc.value_field = key, len(fields) - 1 if value is None else value
        sc.f1_field = -1 if f1 is None else f1
        int_key = fields[key] == "int"
        on_gpu = self.prefix == "fw"
        dev_in = on_gpu and hasattr(data, "is_cuda") and data.is_cuda
        if not dev_in:
            data = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data
        nbytes = int(data.numel() if dev_in else data.size)
        cap = record_cap or max(1, nbytes // 9)
        if on_gpu:
            import torch
            dev = torch.device("cuda", self.cfg.device)
            mk = lambda n, dt=torch.int64: torch.empty(max(n, 1), dtype=dt, device=dev)
            ptr = lambda t: ctypes.c_void_p(t.data_ptr())
        else:
            mk = lambda n, dt=np.int64: np.empty(max(n, 1), dtype=np.int32 if dt is not np.int64 else np.int64)
            ptr = lambda t: ctypes.c_void_p(t.ctypes.data)
        i32 = torch.int32 if on_gpu else np.int32
        if buffers is not None:
            cols = buffers
            if cols["key"].shape[0] < cap or cols["wm"].shape[0] < marker_cap or (int_key and cols["key_hash"] is None):
                raise ValueError("decode buffers smaller than the capacities asked for")
        else:
            cols = dict(key=mk(cap), f1=mk(cap), ts=mk(cap), value=mk(cap), wm=mk(marker_cap), wm_pos=mk(marker_cap),
                        lm=mk(2 * marker_cap), lm_pos=mk(marker_cap))
            cols["key_hash"] = mk(cap, i32) if int_key else None
        src = ctypes.c_void_p(data.data_ptr()) if dev_in else ctypes.c_void_p(data.ctypes.data)
        args = (self.h, ctypes.byref(sc), src, nbytes, _abi.FW_MEM_DEVICE if dev_in else _abi.FW_MEM_HOST,
                ptr(cols["key"]), ptr(cols["key_hash"]) if int_key else None, ptr(cols["f1"]), ptr(cols["ts"]),
                ptr(cols["value"]), cap, ptr(cols["wm"]), ptr(cols["wm_pos"]), ptr(cols["lm"]), ptr(cols["lm_pos"]),
                marker_cap)
        h = dict(cols=cols, data=data, on_gpu=on_gpu, device=device, double=fields[sc.value_field] == "double")
        if on_gpu:
            t = ctypes.c_int32()
            self._check(self._fn("decode_begin")(*args, ctypes.byref(t)))
            h["ticket"] = t.value
        else:   # the oracle decodes synchronously
            cnt = _abi.FwDecodeCounts()
            self._check(self._fn("decode")(*args, ctypes.byref(cnt)))
            h["counts"] = cnt
        return h

    def decode_end(self, h):
        """fw_decode_end of a decode_begin handle: the decoded columns and counts (see decode())."""
        cols = h["cols"]
        if "ticket" in h:
            cnt = _abi.FwDecodeCounts()
            self._check(self._fn("decode_end")(self.h, h["ticket"], ctypes.byref(cnt)))
        else:
            cnt = h["counts"]
        n, nw, nl = cnt.n_records, cnt.n_watermarks, cnt.n_latency_markers
        out = {"n_records": n, "n_watermarks": nw, "n_latency_markers": nl, "consumed": cnt.consumed, "buffers": cols}
        for k in ("key", "key_hash", "f1", "ts", "value"):
            out[k] = None if cols[k] is None else cols[k][:n]
        out["wm"], out["wm_pos"] = cols["wm"][:nw], cols["wm_pos"][:nw]
        out["lm"], out["lm_pos"] = cols["lm"][:2 * nl].reshape(-1, 2), cols["lm_pos"][:nl]
        if h["double"]:
            import torch
            out["value"] = out["value"].view(torch.float64 if h["on_gpu"] else np.float64)
        if h["on_gpu"] and not h["device"]:
            out = {k: (v.cpu().numpy() if hasattr(v, "cpu") else v) for k, v in out.items() if k != "buffers"}
        return out

    def stats(self):
        st = _abi.FwStats()
        self._check(self._fn("get_stats")(self.h, ctypes.byref(st)))
        return {k: getattr(st, k) for k, _ in _abi.FwStats._fields_}

    def close(self):
        if self.h:
            self._fn("destroy")(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


STATE_FIELDS = {"key": _abi.FW_SF_KEY, "f1": _abi.FW_SF_F1, "sum": _abi.FW_SF_SUM, "min": _abi.FW_SF_MIN,
                "max": _abi.FW_SF_MAX, "count": _abi.FW_SF_COUNT, "value": _abi.FW_SF_VALUE}


def state_layout(fields):
    """fw_state_layout of a state tuple given as field names in tuple order, e.g. ("key", "f1", "sum") for
    the Tuple3(key, f1, sum) of Tuple3.of(a.f0, a.f1, a.f2 + b.f2)."""
    if len(fields) > _abi.FW_SF_MAX_FIELDS:
        raise ValueError("state tuple has too many fields")
    L = _abi.FwStateLayout()
    L.n_fields = len(fields)
    for i, f in enumerate(fields):
        L.field[i] = STATE_FIELDS[f]
    return L


def make_config(assigner, reduce_function, trigger=None, allowed_lateness=0, max_parallelism=DEFAULT_MAX_PARALLELISM,
                key_group_range=None, device=0, key_capacity=1 << 16, max_batch=1 << 20, out_capacity=1 << 20,
                max_open_slices=0, ingest_mode=0):
    trigger = trigger if trigger is not None else EventTimeTrigger.create()
    kg = key_group_range if key_group_range is not None else (0, max_parallelism - 1)
    c = _abi.FwConfig()
    c.assigner = assigner.kind
    c.trigger = trigger.code
    c.size = assigner.size
    c.slide = assigner.slide
    c.offset = assigner.offset
    c.allowed_lateness = allowed_lateness
    c.value_type = reduce_function.vt
    c.agg_mask = reduce_function.mask
    c.keep_first_f1 = 1 if reduce_function.keep_first_f1 else 0
    c.max_parallelism = max_parallelism
    c.kg_start, c.kg_end = kg
    c.device = device
    c.max_open_slices = max_open_slices
    c.key_capacity = key_capacity
    c.max_batch = max_batch
    c.out_capacity = out_capacity
    c.ingest_mode = ingest_mode
    c.agg_flags = getattr(reduce_function, "flags", 0)
    c.fold_initial = getattr(reduce_function, "initial_bits", 0)
    c.list_capacity = getattr(reduce_function, "list_capacity", 0)
    return c


class WindowOperator:
    """Event-time WindowOperator (non-merging, reduce) on the GPU.

    processElement(StreamRecord((key, value) | (key, f1, value), ts)) buffers the record;
    processWatermark(Watermark) hands the buffered epoch to the engine, advances the watermark and
    appends the fired results followed by the watermark to the output (AbstractStreamOperator
    .processWatermark :803-808: timers fire, then the watermark is forwarded).
    `window_function`: WindowedStream.reduce(reduceFunction, windowFunction) / apply(reduce, function)
    (WindowedStream.java:347-425): the reduce runs on the GPU, the window function on the host for every
    fired pane, as InternalSingleValueWindowFunction does (InternalSingleValueWindowFunction.java:51-53):
    apply(key, TimeWindow, [reduced value], Collector), each collected element timestamped with
    window.maxTimestamp() (TimestampedCollector, WindowOperator.java:435-438).  A plain callable with the
    same arguments works too.
    `engine_factory(config)` lets the tests run the oracle behind the same surface.
    """

    def __init__(self, assigner, reduce_function, trigger=None, allowed_lateness=0, engine_factory=None,
                 window_function=None, **kw):
        self.assigner = assigner
        self.window_function = window_function
        self.reduce = reduce_function
        self.config = make_config(assigner, reduce_function, trigger, allowed_lateness, **kw)
        self.engine = (engine_factory or WindowEngine)(self.config)
        self._keys, self._hash, self._f1, self._ts, self._val = [], [], [], [], []
        self._key_ids, self._key_names = {}, {}
        self.output = []

    # keys: int (Long) keys pass through with Long.hashCode; String keys are interned to dense ids and
    # carry String.hashCode(), which is what KeyGroupRangeAssignment hashes (KeyGroupRangeAssignment.java:51-64).
    # One operator takes one key type (a keyed stream has one key type), so interned ids never meet Long keys.
    def _key(self, k):
        if isinstance(k, (int, np.integer)) and not isinstance(k, bool):
            if self._key_ids:
                raise TypeError("a keyed stream has one key type: Long key after String keys")
            self._long_keys = True
            return int(k), None
        if not isinstance(k, str):
            raise TypeError(f"key type {type(k).__name__} is not supported (Long or String keys: their Java "
                            "hashCode() decides the key group)")
        if getattr(self, "_long_keys", False):
            raise TypeError("a keyed stream has one key type: String key after Long keys")
        kid = self._key_ids.get(k)
        if kid is None:
            kid = len(self._key_ids) + 1
            self._key_ids[k] = kid
            self._key_names[kid] = k
        return kid, java_string_hash(k)

    def processElement(self, record):
        v = record.value
        self._arity = len(v)
        key, h = self._key(v[0])
        if len(v) == 3:
            f1, val = v[1], v[2]
        else:
            f1, val = record.timestamp, v[1]
        self._keys.append(key)
        self._hash.append(h)
        self._f1.append(f1)
        self._ts.append(record.timestamp)
        self._val.append(val)

    def _flush(self):
        if not self._keys:
            return
        keys = np.array(self._keys, dtype=np.int64)
        hashes = None
        if any(h is not None for h in self._hash):
            from .keygroups import long_hash_code
            hashes = np.array([h if h is not None else long_hash_code(k) for k, h in zip(self._keys, self._hash)],
                              dtype=np.int32)
        ts = np.array(self._ts, dtype=np.int64)
        f1 = np.array(self._f1, dtype=np.int64)
        val = np.array(self._val, dtype=np.int64 if self.reduce.value_type == "i64" else np.float64)
        self._keys, self._hash, self._f1, self._ts, self._val = [], [], [], [], []
        self.engine.push(keys, ts, val, key_hash=hashes, f1=f1)

    def processWatermark(self, mark):
        self._flush()
        self.engine.advance_watermark(mark.timestamp)
        self._drain()

    def _record(self, res, i):
        k = int(res["key"][i])
        key = self._key_names.get(k, k) if self._key_names else k
        vals = []
        if self.reduce.keep_first_f1:
            vals.append(int(res["f1"][i]))
        for f in self.reduce.fields:
            c = ReduceFunction.COLUMN[f]
            col = res[c + ("" if c == "count" else ("_i64" if self.reduce.value_type == "i64" else "_f64"))]
            vals.append(col[i].item())
        ts = int(res["ts"][i])
        value = tuple([key] + vals)
        if self.window_function is None:
            return [StreamRecord(value, ts)]
        out = Collector()
        start = int(res["win_start"][i]) if res.get("win_start") is not None else ts + 1 - self.assigner.size
        window = TimeWindow(start, ts + 1)
        apply = getattr(self.window_function, "apply", self.window_function)
        apply(key, window, [value], out)
        return [StreamRecord(x, ts) for x in out.items]

    def _list_groups(self, res, lo, hi):
        """List state: rows lo..hi are elements grouped by (key, window); the window function gets each group
        (apply(key, TimeWindow, [elements in arrival order], Collector)), or the elements pass through."""
        out = []
        i = lo
        vals = res["sum_i64"] if self.reduce.value_type == "i64" else res["sum_f64"]
        while i < hi:
            k, ts = int(res["key"][i]), int(res["ts"][i])
            j = i
            while j < hi and int(res["key"][j]) == k and int(res["ts"][j]) == ts:
                j += 1
            key = self._key_names.get(k, k) if self._key_names else k
            elems = [(key, int(res["f1"][x]), vals[x].item()) if getattr(self, "_arity", 2) == 3 else
                     (key, vals[x].item()) for x in range(i, j)]
            if self.window_function is None:
                out.extend(StreamRecord(e, ts) for e in elems)
            else:
                col = Collector()
                apply = getattr(self.window_function, "apply", self.window_function)
                start = int(res["win_start"][i]) if res.get("win_start") is not None else ts + 1 - self.assigner.size
                apply(key, TimeWindow(start, ts + 1), elems, col)
                out.extend(StreamRecord(x, ts) for x in col.items)
            i = j
        return out

    def _drain(self):
        res = self.engine.collect()
        if isinstance(self.reduce, ListStateDescriptor):
            pos = 0
            for wm, mp in zip(res["mark_wm"], res["mark_pos"]):
                self.output.extend(self._list_groups(res, pos, int(mp)))
                pos = int(mp)
                self.output.append(Watermark(int(wm)))
            self.output.extend(self._list_groups(res, pos, res["n"]))
            return
        pos = 0
        for wm, mp in zip(res["mark_wm"], res["mark_pos"]):
            while pos < mp:
                self.output.extend(self._record(res, pos))
                pos += 1
            self.output.append(Watermark(int(wm)))
        while pos < res["n"]:
            self.output.extend(self._record(res, pos))
            pos += 1

    def snapshotState(self):
        """{key group: blob} for this subtask's key groups (AbstractStreamOperator.snapshotState
        :367-391 writes the keyed state and the timers of each key group of the local range).  Buffered
        records are handed to the engine first, as the task flushes before the barrier."""
        self._flush()
        if self._key_names:
            raise _abi.FwError(_abi.FW_ERR_UNSUPPORTED, "snapshot needs Long keys")
        lo, hi = self.config.kg_start, self.config.kg_end
        return {kg: self.engine.snapshot_kg(kg) for kg in range(lo, hi + 1)}

    def initializeState(self, state):
        """Restore the blobs of the local key groups (AbstractStreamOperator.initializeState :405-425 reads
        only the key groups of the new range: StateAssignmentOperation hands each subtask its share)."""
        lo, hi = self.config.kg_start, self.config.kg_end
        for kg, blob in sorted(state.items()):
            if lo <= kg <= hi:
                self.engine.restore_kg(kg, blob)

    def getOutput(self):
        return self.output

    def close(self):
        self.engine.close()
