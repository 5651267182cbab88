"""ctypes view of include/flink_window.h and the loader of the HIP engine library.

The product path is libflink_window.so (hand-written HIP for gfx950, built in-tree by
flink_amd.build).  There is no CPU fallback: if the library is missing, loading fails loudly.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# FW_LIBRARY: another build of the same engine (A/B measurements of two builds in one run)
LIB_PATH = os.environ.get("FW_LIBRARY") or os.path.join(HERE, "lib", "libflink_window.so")

# return codes
FW_OK = 0
FW_ERR_INVALID_ARG = 1
FW_ERR_NO_TIMESTAMP = 2
FW_ERR_CAPACITY = 3
FW_ERR_KEY_GROUP = 4
FW_ERR_UNSUPPORTED = 5
FW_ERR_DEVICE = 6

FW_TUMBLING = 0
FW_SLIDING = 1
FW_SESSION = 2
FW_TRIGGER_EVENT_TIME = 0
FW_TRIGGER_PURGING_EVENT_TIME = 1
FW_AGG_SUM = 1
FW_AGG_MIN = 2
FW_AGG_MAX = 4
FW_AGG_COUNT = 8
FW_AGG_MAXBY = 16
FW_AGG_MINBY = 32
FW_AGGF_COMPARABLE = 1
FW_AGGF_BY_LAST = 2
FW_AGGF_FOLD = 4
FW_AGG_LIST = 64
FW_VALUE_I64 = 0
FW_VALUE_F64 = 1
FW_MEM_HOST = 0
FW_MEM_DEVICE = 1

# every entry point include/flink_window.h declares
EXPORTED_SYMBOLS = ("fw_create", "fw_push_batch", "fw_advance_watermark", "fw_sync", "fw_collect",
                    "fw_get_stats", "fw_last_error", "fw_destroy", "fw_partition_by_operator", "fw_partition_by_operator_last", "fw_set_profiling",
                    "fw_get_profile", "fw_debug_counters", "fw_debug_stamps", "fw_set_stream", "fw_stream_wait_input",
                    "fw_version", "fw_snapshot_kg", "fw_restore_kg", "fw_snapshot_kg_flink", "fw_restore_kg_flink", "fw_decode",
                    "fw_collect_begin", "fw_collect_end", "fw_decode_begin", "fw_decode_end")
FW_SNAP_MAGIC, FW_SNAP_HEADER_WORDS, FW_SNAP_ENTRY_WORDS = 0x31474b5746574b, 14, 8
# state tuple fields of the Flink-layout checkpoint (fw_state_layout)
FW_SF_KEY, FW_SF_F1, FW_SF_SUM, FW_SF_MIN, FW_SF_MAX, FW_SF_COUNT, FW_SF_VALUE, FW_SF_MAX_FIELDS = 1, 2, 3, 4, 5, 6, 7, 8
FW_FT_LONG, FW_FT_DOUBLE, FW_FT_INT = 0, 1, 2
FW_PHASE_INGEST, FW_PHASE_FIXUP, FW_PHASE_LATE, FW_PHASE_FIRE, FW_PHASE_AGGREGATE, FW_NPHASES = 0, 1, 2, 3, 4, 5

_i32, _i64, _p = ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p
_pi64 = ctypes.POINTER(ctypes.c_int64)
_pf64 = ctypes.POINTER(ctypes.c_double)


class FwConfig(ctypes.Structure):
    _fields_ = [("assigner", _i32), ("trigger", _i32), ("size", _i64), ("slide", _i64), ("offset", _i64),
                ("allowed_lateness", _i64), ("value_type", _i32), ("agg_mask", _i32), ("keep_first_f1", _i32),
                ("max_parallelism", _i32), ("kg_start", _i32), ("kg_end", _i32), ("device", _i32),
                ("max_open_slices", _i32), ("key_capacity", _i64), ("max_batch", _i64), ("out_capacity", _i64),
                ("ingest_mode", _i32), ("agg_flags", _i32), ("fold_initial", _i64),
                ("list_capacity", _i64)]


class FwOut(ctypes.Structure):
    _fields_ = [("n", _i64), ("key", _pi64), ("f1", _pi64), ("ts", _pi64), ("sum_i64", _pi64), ("min_i64", _pi64),
                ("max_i64", _pi64), ("count", _pi64), ("sum_f64", _pf64), ("min_f64", _pf64), ("max_f64", _pf64),
                ("n_marks", _i64), ("mark_wm", _pi64), ("mark_pos", _pi64), ("win_start", _pi64)]


class FwStateLayout(ctypes.Structure):
    _fields_ = [("n_fields", _i32), ("field", _i32 * FW_SF_MAX_FIELDS)]


class FwTupleSchema(ctypes.Structure):
    _fields_ = [("n_fields", _i32), ("field_type", _i32 * 8), ("key_field", _i32), ("f1_field", _i32),
                ("value_field", _i32)]


class FwDecodeCounts(ctypes.Structure):
    _fields_ = [("n_records", _i64), ("n_watermarks", _i64), ("n_latency_markers", _i64), ("consumed", _i64)]


class FwProfile(ctypes.Structure):
    _fields_ = [("ms", ctypes.c_double * FW_NPHASES), ("launches", _i64 * FW_NPHASES), ("records", _i64 * FW_NPHASES)]


class FwStats(ctypes.Structure):
    _fields_ = [("records_in", _i64), ("records_late", _i64), ("panes_fired", _i64), ("late_fires", _i64),
                ("keys_resident", _i64), ("slices_live", _i64), ("ingest_form", _i64), ("compactions", _i64)]


def declare(lib, prefix="fw"):
    """Attach argtypes/restypes for the fw_* (or fwo_* oracle) entry points present in `lib`."""
    P = ctypes.POINTER
    sigs = {
        "create": (_i32, [P(FwConfig), P(_p)]),
        "push_batch": (_i32, [_p, _p, _p, _p, _p, _p, _i64] + ([_i32] if prefix == "fw" else [])),
        "advance_watermark": (_i32, [_p, _i64]),
        "sync": (_i32, [_p]),
        "collect": (_i32, [_p, P(FwOut)] + ([_i32] if prefix == "fw" else [])),
        "collect_begin": (_i32, [_p, P(_i32)]),
        "collect_end": (_i32, [_p, _i32, P(FwOut)]),
        "get_stats": (_i32, [_p, P(FwStats)]),
        "last_error": (ctypes.c_char_p, [_p]),
        "destroy": (None, [_p]),
        "partition_by_operator": (_i32, [_p, _p, _p, _p, _p, _p, _i64, _i32, _i32, _p, _p, _p, _p, _p, _p, _p]),
        "partition_by_operator_last": (_i32, [_p, _p, _p, _p, _p, _p, _i64, _i32, _i32, _p, _p, _p, _p, _p, _p, _p, _i32]),
        "version": (ctypes.c_char_p, []),
        "set_profiling": (_i32, [_p, _i32]),
        "get_profile": (_i32, [_p, P(FwProfile)]),
        "debug_counters": (_i32, [_p, _p]),
        "set_stream": (_i32, [_p, _p]),
        "stream_wait_input": (_i32, [_p, _p, _i32]),
        "snapshot_kg": (_i32, [_p, _i32, _p, _i64, P(_i64)]),
        "restore_kg": (_i32, [_p, _i32, _p, _i64]),
        "snapshot_kg_flink": (_i32, [_p, _i32, P(FwStateLayout), _p, _i64, P(_i64), _p, _i64, P(_i64)]),
        "restore_kg_flink": (_i32, [_p, _i32, P(FwStateLayout), _i64, _p, _i64, _p, _i64]),
        "decode": (_i32, [_p, P(FwTupleSchema), _p, _i64, _i32, _p, _p, _p, _p, _p, _i64, _p, _p, _p, _p, _i64,
                          P(FwDecodeCounts)]),
        "decode_begin": (_i32, [_p, P(FwTupleSchema), _p, _i64, _i32, _p, _p, _p, _p, _p, _i64, _p, _p, _p, _p, _i64,
                                P(_i32)]),
        "decode_end": (_i32, [_p, _i32, P(FwDecodeCounts)]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(lib, f"{prefix}_{name}", None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
    return lib


_lib = None


def open_library(path):
    if not os.path.exists(path):
        raise RuntimeError(f"HIP engine library not built: {path} (run flink_amd.build.build_all())")
    return declare(ctypes.CDLL(path), "fw")


def load_library():
    """Load libflink_window.so (no fallback: a missing library is an error)."""
    global _lib
    if _lib is None:
        # torch bundles its own HIP runtime; it has to initialise before the engine's (the image's ROCm) does,
        # or torch finds no GPU later in the same process.  The engine itself does not use torch.
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.init()
        except ImportError:
            pass
        _lib = open_library(LIB_PATH)
    return _lib


class FwError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[fw error {code}] {msg}")
        self.code = code
