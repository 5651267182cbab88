"""KeyGroupRangeAssignment for the host side (routing math, key-group ranges), Java semantics.

Mirrors flink-runtime/src/main/java/org/apache/flink/runtime/state/KeyGroupRangeAssignment.java
(:26 DEFAULT_MAX_PARALLELISM, :40-42 assignKeyToParallelOperator, :51-53 assignToKeyGroup,
:62-64 computeKeyGroupForKeyHash, :78-89 computeKeyGroupRangeForOperatorIndex,
:105-107 computeOperatorIndexForKeyGroup) and MathUtils.murmurHash
(flink-core/src/main/java/org/apache/flink/util/MathUtils.java:134-158).
The device computes the same functions per record (flink_amd/csrc/java_semantics.h); these host
versions size key-group ranges per GPU and route records in the CPU (gloo) exchange tests.
"""
import numpy as np

DEFAULT_MAX_PARALLELISM = 128


def _i32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= (1 << 31) else x


def murmur_hash(code):
    """MathUtils.murmurHash(int)."""
    c = code & 0xFFFFFFFF
    c = (c * 0xCC9E2D51) & 0xFFFFFFFF
    c = ((c << 15) | (c >> 17)) & 0xFFFFFFFF
    c = (c * 0x1B873593) & 0xFFFFFFFF
    c = ((c << 13) | (c >> 19)) & 0xFFFFFFFF
    c = (c * 5 + 0xE6546B64) & 0xFFFFFFFF
    c ^= 4
    c ^= c >> 16
    c = (c * 0x85EBCA6B) & 0xFFFFFFFF
    c ^= c >> 13
    c = (c * 0xC2B2AE35) & 0xFFFFFFFF
    c ^= c >> 16
    code = _i32(c)
    if code >= 0:
        return code
    if code != -(1 << 31):
        return -code
    return 0


def long_hash_code(v):
    """JDK Long.hashCode(long): (int)(v ^ (v >>> 32))."""
    u = v & 0xFFFFFFFFFFFFFFFF
    return _i32((u ^ (u >> 32)) & 0xFFFFFFFF)


def compute_key_group_for_key_hash(key_hash, max_parallelism):
    return murmur_hash(key_hash) % max_parallelism


def assign_to_key_group(key, max_parallelism, key_hash=None):
    return compute_key_group_for_key_hash(long_hash_code(key) if key_hash is None else key_hash, max_parallelism)


def compute_operator_index_for_key_group(max_parallelism, parallelism, key_group):
    return key_group * parallelism // max_parallelism


def assign_key_to_parallel_operator(key, max_parallelism, parallelism, key_hash=None):
    return compute_operator_index_for_key_group(max_parallelism, parallelism,
                                                assign_to_key_group(key, max_parallelism, key_hash))


def compute_key_group_range_for_operator_index(max_parallelism, parallelism, operator_index):
    if parallelism <= 0:
        raise ValueError("Parallelism must not be smaller than zero.")
    if max_parallelism < parallelism:
        raise ValueError("Maximum parallelism must not be smaller than parallelism.")
    if max_parallelism > (1 << 15):
        raise ValueError("Maximum parallelism must be smaller than 2^15.")
    start = 0 if operator_index == 0 else ((operator_index * max_parallelism - 1) // parallelism) + 1
    end = ((operator_index + 1) * max_parallelism - 1) // parallelism
    return start, end


# ---- vectorised (numpy) forms for the host routing of whole batches ----
def murmur_hash_np(code):
    c = np.asarray(code).astype(np.int64).astype(np.uint32)
    with np.errstate(over="ignore"):
        c = c * np.uint32(0xCC9E2D51)
        c = (c << np.uint32(15)) | (c >> np.uint32(17))
        c = c * np.uint32(0x1B873593)
        c = (c << np.uint32(13)) | (c >> np.uint32(19))
        c = c * np.uint32(5) + np.uint32(0xE6546B64)
        c ^= np.uint32(4)
        c ^= c >> np.uint32(16)
        c = c * np.uint32(0x85EBCA6B)
        c ^= c >> np.uint32(13)
        c = c * np.uint32(0xC2B2AE35)
        c ^= c >> np.uint32(16)
    s = c.view(np.int32).astype(np.int64)
    return np.where(s >= 0, s, np.where(s != -(1 << 31), -s, 0))


def long_hash_code_np(keys):
    u = np.asarray(keys, dtype=np.int64).view(np.uint64)
    return ((u ^ (u >> np.uint64(32))) & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32)


def operator_index_np(keys, max_parallelism, parallelism, key_hash=None):
    h = long_hash_code_np(keys) if key_hash is None else np.asarray(key_hash, dtype=np.int32)
    kg = murmur_hash_np(h) % max_parallelism
    return (kg * parallelism // max_parallelism).astype(np.int64)
