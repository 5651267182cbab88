"""Generate the golden fixtures under tests/golden/ from the reference's own tests.

Every expected output below is transcribed from the reference test that states it (file:line,
paths relative to the reference root; WOT = flink-streaming-java/src/test/java/org/apache/flink/
streaming/runtime/operators/windowing/WindowOperatorTest.java).  Nothing here runs the reference
(there is no JVM in the image) and nothing here runs the oracle: the fixtures pin the oracle.

String keys of the reference tests are mapped to int64 key ids; their Java String.hashCode() is
carried per event (the key group of a String key comes from its hashCode, KeyGroupRangeAssignment
.assignToKeyGroup:51-53).  Integer values (Tuple2<String,Integer>, SumReducer WOT:2245-2252) are
small, so an int64 sum gives the same results.

Run:  python tests/golden/make_fixtures.py   (rewrites the *.json files next to this script)
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LONG_MAX = (1 << 63) - 1


def java_string_hash(s):
    """java.lang.String.hashCode(): s[0]*31^(n-1) + ... + s[n-1], int32 wrapping."""
    h = 0
    for ch in s:
        h = (31 * h + ord(ch)) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


KEYS = {"key1": 1, "key2": 2}
KEY_HASH = {KEYS[k]: java_string_hash(k) for k in KEYS}


def rec(key, value, ts):
    return ["rec", KEYS[key], value, ts]


def wm(t):
    return ["wm", t]


def out(key, value, ts):
    return [KEYS[key], value, ts]


def cfg(assigner, size, slide=0, offset=0, lateness=0, trigger="event_time"):
    return {"assigner": assigner, "size": size, "slide": slide, "offset": offset,
            "allowed_lateness": lateness, "trigger": trigger, "value_type": "i64", "agg": ["sum"],
            "keep_first_f1": False, "max_parallelism": 1}


def fixture(name, source, config, events, expected):
    return {"name": name, "source": source, "config": config, "key_hash": {str(k): v for k, v in KEY_HASH.items()},
            "events": events, "expected": expected}


# elements common to the sliding/tumbling reduce tests, WOT:95-105 and WOT:200-210
OOO_ELEMENTS = [rec("key2", 1, 3999), rec("key2", 1, 3000), rec("key1", 1, 20), rec("key1", 1, 0),
                rec("key1", 1, 999), rec("key2", 1, 1998), rec("key2", 1, 1999), rec("key2", 1, 1000)]

FIXTURES = []

# WOT:92-157 testSlidingEventTimeWindows (size 3s, slide 1s), reduce variant :161-192.
# (the mid-stream snapshot/restore of the reference test keeps state, so results are unchanged)
FIXTURES.append(fixture(
    "sliding_reduce", "WindowOperatorTest.java:92-192",
    cfg("sliding", 3000, 1000),
    OOO_ELEMENTS + [wm(999), wm(1999), wm(2999), wm(3999), wm(4999), wm(5999), wm(6999), wm(7999)],
    [{"wm": 999, "records": [out("key1", 3, 999)]},
     {"wm": 1999, "records": [out("key1", 3, 1999), out("key2", 3, 1999)]},
     {"wm": 2999, "records": [out("key1", 3, 2999), out("key2", 3, 2999)]},
     {"wm": 3999, "records": [out("key2", 5, 3999)]},
     {"wm": 4999, "records": [out("key2", 2, 4999)]},
     {"wm": 5999, "records": [out("key2", 2, 5999)]},
     {"wm": 6999, "records": []},
     {"wm": 7999, "records": []}]))

# WOT:196-263 testTumblingEventTimeWindows (size 3s), reduce variant :267-298
FIXTURES.append(fixture(
    "tumbling_reduce", "WindowOperatorTest.java:196-298",
    cfg("tumbling", 3000),
    OOO_ELEMENTS + [wm(999), wm(1999), wm(2999), wm(3999), wm(4999), wm(5999), wm(6999), wm(7999)],
    [{"wm": 999, "records": []},
     {"wm": 1999, "records": []},
     {"wm": 2999, "records": [out("key1", 3, 2999), out("key2", 3, 2999)]},
     {"wm": 3999, "records": []},
     {"wm": 4999, "records": []},
     {"wm": 5999, "records": [out("key2", 2, 5999)]},
     {"wm": 6999, "records": []},
     {"wm": 7999, "records": []}]))

# WOT:1106-1161 testLateness: tumbling 2s, PurgingTrigger(EventTimeTrigger), lateness 500
FIXTURES.append(fixture(
    "lateness_purging", "WindowOperatorTest.java:1106-1161",
    cfg("tumbling", 2000, lateness=500, trigger="purging_event_time"),
    [rec("key2", 1, 500), wm(1500), rec("key2", 1, 1300), wm(2300), rec("key2", 1, 1997), wm(6000),
     rec("key2", 1, 1998), wm(7000)],
    [{"wm": 1500, "records": []},
     {"wm": 2300, "records": [out("key2", 2, 1999)]},
     {"wm": 6000, "records": [out("key2", 1, 1999)]},
     {"wm": 7000, "records": []}]))

# WOT:1164-1229 testCleanupTimeOverflow: tumbling 1000 ms, lateness 2000, ts = Long.MAX_VALUE - 1750
_ts = LONG_MAX - 1750
_start = _ts - (_ts - 0 + 1000) % 1000  # TimeWindow.getWindowStartWithOffset (no overflow here)
_max_ts = _start + 1000 - 1
FIXTURES.append(fixture(
    "cleanup_time_overflow", "WindowOperatorTest.java:1164-1229",
    cfg("tumbling", 1000, lateness=2000),
    [rec("key2", 1, _ts), wm(LONG_MAX - 1500), wm(_max_ts)],
    [{"wm": LONG_MAX - 1500, "records": []},
     {"wm": _max_ts, "records": [out("key2", 1, _max_ts)]}]))

# WOT:1232-1288 testDropDueToLatenessTumbling: tumbling 2s, lateness 0
FIXTURES.append(fixture(
    "drop_late_tumbling", "WindowOperatorTest.java:1232-1288",
    cfg("tumbling", 2000),
    [rec("key2", 1, 1000), wm(1985), rec("key2", 1, 1980), wm(1999), rec("key2", 1, 1998),
     rec("key2", 1, 2001), wm(2999), wm(3999)],
    [{"wm": 1985, "records": []},
     {"wm": 1999, "records": [out("key2", 2, 1999)]},
     {"wm": 2999, "records": []},
     {"wm": 3999, "records": [out("key2", 1, 3999)]}]))

# WOT:1291-1364 testDropDueToLatenessSliding: sliding 3s/1s, lateness 0
FIXTURES.append(fixture(
    "drop_late_sliding", "WindowOperatorTest.java:1291-1364",
    cfg("sliding", 3000, 1000),
    [rec("key2", 1, 1000), wm(1999), rec("key2", 1, 2000), wm(3000), rec("key1", 1, 3001),
     rec("key2", 1, 2400), rec("key2", 1, 2400), rec("key1", 1, 3001), rec("key2", 1, 3900), wm(6000),
     rec("key1", 1, 3001), wm(25000)],
    [{"wm": 1999, "records": [out("key2", 1, 1999)]},
     {"wm": 3000, "records": [out("key2", 2, 2999)]},
     {"wm": 6000, "records": [out("key2", 5, 3999), out("key1", 2, 3999), out("key2", 4, 4999),
                              out("key1", 2, 4999), out("key2", 1, 5999), out("key1", 2, 5999)]},
     {"wm": 25000, "records": []}]))

# WOT:1988-2032 testCleanupTimerWithEmptyReduceStateForTumblingWindows: tumbling 2s, lateness 1
FIXTURES.append(fixture(
    "cleanup_timer_empty_state", "WindowOperatorTest.java:1988-2032",
    cfg("tumbling", 2000, lateness=1),
    [rec("key2", 1, 1000), wm(1599), wm(1999), wm(2000), wm(5000)],
    [{"wm": 1599, "records": []},
     {"wm": 1999, "records": [out("key2", 1, 1999)]},
     {"wm": 2000, "records": []},
     {"wm": 5000, "records": []}]))

# WOT:2467-2505 testEventTimeTumblingWindowsWithOffset: size 2000, offset 100.  The reference test
# emits the window's elements one by one (a list window function); with the reduce (sum) the same
# window [100, 2100) yields one record 1+2+3+4 = 10 at maxTimestamp 2099.
FIXTURES.append(fixture(
    "tumbling_offset", "WindowOperatorTest.java:2467-2505 (window contents summed)",
    cfg("tumbling", 2000, offset=100),
    [rec("key2", 1, 1000), wm(1985), rec("key2", 2, 1980), rec("key2", 3, 1998), rec("key2", 4, 2001),
     wm(2010), wm(2999), wm(3999)],
    [{"wm": 1985, "records": []},
     {"wm": 2010, "records": []},
     {"wm": 2999, "records": [out("key2", 10, 2099)]},
     {"wm": 3999, "records": []}]))

# WOT:2508-2541 testEventTimeSlidingWindowsWithOffset: size 2000, slide 500, offset 10
FIXTURES.append(fixture(
    "sliding_offset", "WindowOperatorTest.java:2508-2541",
    cfg("sliding", 2000, 500, offset=10),
    [rec("key2", 1, 333), wm(6666)],
    [{"wm": 6666, "records": [out("key2", 1, 509), out("key2", 1, 1009), out("key2", 1, 1509),
                              out("key2", 1, 2009)]}]))


# HAND-DERIVED (no reference test runs sliding windows with allowed lateness > 0): WOT:1104-1161
# testLateness's input over SlidingEventTimeWindows.of(3 s, 1 s), lateness 500, SumReducer, worked out
# step by step from WindowOperator.processElement / onEventTime (WindowOperator.java:302-375, isLate
# :470-472, cleanupTime :511-514), EventTimeTrigger (:37-52) and PurgingTrigger (:47-55):
#  500   -> windows [0,3000) [-1000,2000) [-2000,1000)
#  wm 1500  fires [-2000,1000) = 1 @999 (cleanup 1499 passes too)
#  1300  -> [1000,4000) [0,3000) [-1000,2000), none late, none fires (all maxTs > 1500)
#  wm 2300  fires [-1000,2000) = 2 @1999
#  1997  -> same three windows, none late (cleanups 2499/3499/4499 > 2300); [-1000,2000) has maxTs
#           1999 <= 2300: the element FIRES it -> 3 (accumulating), or 1 (purging: the watermark fire
#           purged it, so it holds only this element)
#  wm 6000  cleanup of [-1000,2000) (no output), fires [0,3000) = 3 @2999, [1000,4000) = 2 @3999
#  1998  -> all three windows late (cleanup <= 6000): dropped;  wm 7000 nothing
_SL_EVENTS = [rec("key2", 1, 500), wm(1500), rec("key2", 1, 1300), wm(2300), rec("key2", 1, 1997), wm(6000),
              rec("key2", 1, 1998), wm(7000)]
FIXTURES.append(fixture(
    "sliding_lateness", "hand-derived: WindowOperatorTest.java:1104-1161 inputs, sliding 3s/1s, lateness 500, EventTimeTrigger",
    cfg("sliding", 3000, 1000, lateness=500),
    _SL_EVENTS,
    [{"wm": 1500, "records": [out("key2", 1, 999)]},
     {"wm": 2300, "records": [out("key2", 2, 1999)]},
     {"wm": 6000, "records": [out("key2", 3, 1999), out("key2", 3, 2999), out("key2", 2, 3999)]},
     {"wm": 7000, "records": []}]))
FIXTURES.append(fixture(
    "sliding_lateness_purging", "hand-derived: WindowOperatorTest.java:1104-1161 inputs, sliding 3s/1s, lateness 500, PurgingTrigger",
    cfg("sliding", 3000, 1000, lateness=500, trigger="purging_event_time"),
    _SL_EVENTS,
    [{"wm": 1500, "records": [out("key2", 1, 999)]},
     {"wm": 2300, "records": [out("key2", 2, 1999)]},
     {"wm": 6000, "records": [out("key2", 1, 1999), out("key2", 3, 2999), out("key2", 2, 3999)]},
     {"wm": 7000, "records": []}]))


def closed_form(name, source, size, slide):
    """EventTimeWindowCheckpointingITCase (flink-tests/.../test/checkpointing/...): FailingSource
    :495-579 emits, for next = 0..2999, (key i, next) @ ts=next for keys 0..99, then Watermark(next);
    ValidatingSink :582-686 requires every fired window (key, [start, end)) to hold
    sum_{i=start}^{end-1, i>0} i.  Long keys (keyBy(0) -> Tuple1<Long>.hashCode = Long.hashCode)."""
    n_keys, n_elem = 100, 3000
    config = cfg("tumbling" if slide == 0 else "sliding", size, slide)
    config["max_parallelism"] = 128
    expected = []
    # windows fire when the watermark reaches their maxTimestamp = end - 1
    starts = set()
    step = size if slide == 0 else slide
    for t in range(n_elem):
        last = t - (t + step) % step
        s = last
        while s > t - size:
            starts.add(s)
            s -= step
    by_wm = {}
    for s in starts:
        max_ts = s + size - 1
        if max_ts <= n_elem - 1:
            total = sum(i for i in range(s, s + size) if i > 0)
            total = ((total + (1 << 31)) % (1 << 32)) - (1 << 31)
            by_wm.setdefault(max_ts, []).extend([k, total, max_ts] for k in range(n_keys))
    for t in range(n_elem):
        expected.append({"wm": t, "records": sorted(by_wm.get(t, []))})
    return {"name": name, "source": source, "config": config, "key_hash": {},
            "generator": {"kind": "itcase_failing_source", "n_keys": n_keys, "n_elements": n_elem},
            "expected": expected}


FIXTURES.append(closed_form("itcase_tumbling_closed_form",
                            "EventTimeWindowCheckpointingITCase.java:344-410,495-686", 100, 0))
FIXTURES.append(closed_form("itcase_sliding_closed_form",
                            "EventTimeWindowCheckpointingITCase.java:416-485,495-686", 1000, 100))

# ---- session windows (EventTimeSessionWindows.withGap, the merging branch of WindowOperator) ----
# Expected records carry the window: [key, sum, maxTimestamp, window start].  The reference's
# ReducedSessionWindowFunction / SessionWindowFunction emit Tuple3(key + "-" + sum, window.getStart(),
# window.getEnd()) timestamped window.maxTimestamp() (WOT:2290-2320), i.e. exactly (key, sum, start, end = ts + 1).
def sout(key, value, start, end):
    return [KEYS[key], value, end - 1, start]


SESSION_OOO = [rec("key2", 1, 0), rec("key2", 2, 1000), rec("key2", 3, 2500),
               rec("key1", 1, 10), rec("key1", 2, 1000), rec("key1", 3, 2500),
               rec("key2", 4, 5501), rec("key2", 5, 6000), rec("key2", 5, 6000), rec("key2", 6, 6050)]
SESSION_OUT = [{"wm": 12000, "records": [sout("key1", 6, 10, 5500), sout("key2", 6, 0, 5500), sout("key2", 20, 5501, 9050)]},
               {"wm": 17999, "records": [sout("key2", 30, 15000, 18000)]}]

# WOT:435-501 testReduceSessionWindows (gap 3 s; its mid-stream snapshot/restore keeps the state)
FIXTURES.append(fixture(
    "session_reduce", "WindowOperatorTest.java:435-501", cfg("session", 3000),
    SESSION_OOO + [wm(12000), rec("key2", 10, 15000), rec("key2", 20, 15000), wm(17999)], SESSION_OUT))
# WOT:362-431 testSessionWindows: the same elements through ListState (ListStateDescriptor) +
# SessionWindowFunction, which emits (key-sum, start, end) over the merged window's element list; the replay
# applies that window function to the list-state rows
SESSION_LIST = cfg("session", 3000)
SESSION_LIST["list"] = True
FIXTURES.append(fixture(
    "session_windows", "WindowOperatorTest.java:362-431", SESSION_LIST,
    SESSION_OOO + [wm(12000), rec("key2", 10, 15000), rec("key2", 20, 15000), wm(17999)], SESSION_OUT))


def late_session_events(extra):
    """The common prefix of the testDropDueToLatenessSession* tests (WOT:1395-1417 and its copies)."""
    return [rec("key2", 1, 1000), wm(1999), rec("key2", 1, 2000), wm(4998),
            rec("key2", 1, 4500), rec("key2", 1, 8500), wm(7400),
            rec("key2", 1, 7000), wm(11501),
            rec("key2", 1, 11600), wm(14600)] + extra


LATE_SESSION_PREFIX = [{"wm": 1999, "records": []}, {"wm": 4998, "records": []}, {"wm": 7400, "records": []},
                       {"wm": 11501, "records": [sout("key2", 5, 1000, 11500)]},
                       {"wm": 14600, "records": [sout("key2", 1, 11600, 14600)]}]

# WOT:1367-1448 testDropDueToLatenessSessionZeroLatenessPurgingTrigger
FIXTURES.append(fixture(
    "session_late_zero_purging", "WindowOperatorTest.java:1367-1448",
    cfg("session", 3000, lateness=0, trigger="purging"),
    late_session_events([rec("key2", 1, 10000), rec("key2", 1, 10100), rec("key2", 1, 14500), wm(20000), wm(100000)]),
    LATE_SESSION_PREFIX + [{"wm": 20000, "records": [sout("key2", 1, 14500, 17500)]}, {"wm": 100000, "records": []}]))
# WOT:1451-1534 testDropDueToLatenessSessionZeroLateness
FIXTURES.append(fixture(
    "session_late_zero", "WindowOperatorTest.java:1451-1534", cfg("session", 3000, lateness=0),
    late_session_events([rec("key2", 1, 10000), rec("key2", 1, 14500), wm(20000), wm(100000)]),
    LATE_SESSION_PREFIX + [{"wm": 20000, "records": [sout("key2", 1, 14500, 17500)]}, {"wm": 100000, "records": []}]))
# WOT:1537-1618 testDropDueToLatenessSessionWithLatenessPurgingTrigger (lateness 10)
FIXTURES.append(fixture(
    "session_late_small_purging", "WindowOperatorTest.java:1537-1618",
    cfg("session", 3000, lateness=10, trigger="purging"),
    late_session_events([rec("key2", 1, 10000), rec("key2", 1, 14500), wm(20000), wm(100000)]),
    LATE_SESSION_PREFIX + [{"wm": 20000, "records": [sout("key2", 1, 14500, 17500)]}, {"wm": 100000, "records": []}]))
# WOT:1621-1714 testDropDueToLatenessSessionWithLateness (lateness 10): 10000 merges into the fired
# (11600, 14600) session and fires it at once as (10000, 14600), then 14500 extends it
FIXTURES.append(fixture(
    "session_late_small", "WindowOperatorTest.java:1621-1714", cfg("session", 3000, lateness=10),
    late_session_events([rec("key2", 1, 10000), rec("key2", 1, 14500), wm(20000), wm(100000)]),
    LATE_SESSION_PREFIX + [{"wm": 20000, "records": [sout("key2", 2, 10000, 14600), sout("key2", 3, 10000, 17500)]},
                           {"wm": 100000, "records": []}]))
# WOT:1717-1800 testDropDueToLatenessSessionWithHugeLatenessPurgingTrigger (lateness 10000)
FIXTURES.append(fixture(
    "session_late_huge_purging", "WindowOperatorTest.java:1717-1800",
    cfg("session", 3000, lateness=10000, trigger="purging"),
    late_session_events([rec("key2", 1, 10000), rec("key2", 1, 14500), wm(20000), wm(100000)]),
    LATE_SESSION_PREFIX + [{"wm": 20000, "records": [sout("key2", 1, 10000, 13000), sout("key2", 1, 14500, 17500)]},
                           {"wm": 100000, "records": []}]))
# WOT:1803-1866 testDropDueToLatenessSessionWithHugeLateness (lateness 10000): 10000 bridges the two fired
# sessions into (1000, 14600), which fires at once; 14500 extends it to (1000, 17500)
FIXTURES.append(fixture(
    "session_late_huge", "WindowOperatorTest.java:1803-1866", cfg("session", 3000, lateness=10000),
    late_session_events([rec("key2", 1, 10000), rec("key2", 1, 14500), wm(20000), wm(100000)]),
    LATE_SESSION_PREFIX + [{"wm": 20000, "records": [sout("key2", 7, 1000, 14600), sout("key2", 8, 1000, 17500)]},
                           {"wm": 100000, "records": []}]))
# WOT:2133-2175 testCleanupTimerWithEmptyReduceStateForSessionWindows (gap 3 s, lateness 10)
FIXTURES.append(fixture(
    "session_cleanup_timer", "WindowOperatorTest.java:2133-2175", cfg("session", 3000, lateness=10),
    [rec("key2", 1, 1000), wm(4998), wm(14600)],
    [{"wm": 4998, "records": [sout("key2", 1, 1000, 4000)]}, {"wm": 14600, "records": []}]))

# WOT:2034-2089 testCleanupTimerWithEmptyFoldingStateForTumblingWindows: tumbling 2 s, lateness 1, a
# FoldingStateDescriptor with default (null, 0) and fold (acc, v) -> (v.f0, acc.f1 + v.f1), i.e. a sum from 0
FOLD_CFG = cfg("tumbling", 2000, lateness=1)
FOLD_CFG["fold"] = {"kind": "sum", "initial": 0}
FIXTURES.append(fixture(
    "fold_cleanup_timer", "WindowOperatorTest.java:2034-2089", FOLD_CFG,
    [rec("key2", 1, 1000), wm(1599), wm(1999), wm(2000), wm(5000)],
    [{"wm": 1599, "records": []}, {"wm": 1999, "records": [out("key2", 1, 1999)]}, {"wm": 2000, "records": []},
     {"wm": 5000, "records": []}]))

# ---- list state: WindowedStream.apply(WindowFunction) over ListStateDescriptor (HeapListState) ----
# testSlidingEventTimeWindowsApply / testTumblingEventTimeWindowsApply run the reduce tests' elements through
# list state and RichSumReducer (a window function summing the iterable: WOT:2255-2285), so the expected
# outputs are the reduce tests' (WOT:92-157, WOT:196-263); the replay applies that window function
LIST_SLIDING = cfg("sliding", 3000, 1000)
LIST_SLIDING["list"] = True
FIXTURES.append(fixture(
    "list_sliding_apply", "WindowOperatorTest.java:194-226 (elements/expectations :92-157)", LIST_SLIDING,
    OOO_ELEMENTS + [wm(999), wm(1999), wm(2999), wm(3999), wm(4999), wm(5999), wm(6999), wm(7999)],
    [{"wm": 999, "records": [out("key1", 3, 999)]},
     {"wm": 1999, "records": [out("key1", 3, 1999), out("key2", 3, 1999)]},
     {"wm": 2999, "records": [out("key1", 3, 2999), out("key2", 3, 2999)]},
     {"wm": 3999, "records": [out("key2", 5, 3999)]},
     {"wm": 4999, "records": [out("key2", 2, 4999)]},
     {"wm": 5999, "records": [out("key2", 2, 5999)]},
     {"wm": 6999, "records": []},
     {"wm": 7999, "records": []}]))
LIST_TUMBLING = cfg("tumbling", 3000)
LIST_TUMBLING["list"] = True
FIXTURES.append(fixture(
    "list_tumbling_apply", "WindowOperatorTest.java:326-358 (elements/expectations :196-263)", LIST_TUMBLING,
    OOO_ELEMENTS + [wm(999), wm(1999), wm(2999), wm(3999), wm(4999), wm(5999), wm(6999), wm(7999)],
    [{"wm": 999, "records": []},
     {"wm": 1999, "records": []},
     {"wm": 2999, "records": [out("key1", 3, 2999), out("key2", 3, 2999)]},
     {"wm": 3999, "records": []},
     {"wm": 4999, "records": []},
     {"wm": 5999, "records": [out("key2", 2, 5999)]},
     {"wm": 6999, "records": []},
     {"wm": 7999, "records": []}]))
# WOT:1942-1975 testCleanupTimerWithEmptyListStateForTumblingWindows (tumbling 2 s, lateness 1, the elements
# passed through: one element (key2, 1) -> (key2, 1) @1999)
LIST_CLEANUP = cfg("tumbling", 2000, lateness=1)
LIST_CLEANUP["list"] = True
FIXTURES.append(fixture(
    "list_cleanup_timer", "WindowOperatorTest.java:1942-1976", LIST_CLEANUP,
    [rec("key2", 1, 1000), wm(1599), wm(1999), wm(2000), wm(5000)],
    [{"wm": 1599, "records": []}, {"wm": 1999, "records": [out("key2", 1, 1999)]}, {"wm": 2000, "records": []},
     {"wm": 5000, "records": []}]))

# TimeWindowTest.java:30-58 getWindowStartWithOffset known answers: (ts, offset, size, expected)
WINDOW_START = {
    "source": "flink-streaming-java/src/test/java/org/apache/flink/streaming/runtime/operators/windowing/TimeWindowTest.java:30-58",
    "cases": [[1, 0, 7, 0], [6, 0, 7, 0], [7, 0, 7, 7], [8, 0, 7, 7],
              [1, 3, 7, -4], [2, 3, 7, -4], [3, 3, 7, 3], [9, 3, 7, 3], [10, 3, 7, 10],
              [1, -2, 7, -2], [-2, -2, 7, -2], [3, -2, 7, -2], [4, -2, 7, -2], [7, -2, 7, 5], [12, -2, 7, 12],
              [1470902048450, -8 * 3600 * 1000, 24 * 3600 * 1000, 1470844800000]],
}

# SURVEY.md Appendix B — values computed by an independent MurmurHash3_x86_32 restatement (the
# reference has NO murmur known-answer test; these are a cross-check, not reference output).
MURMUR = {
    "source": "SURVEY.md Appendix B (restatement cross-check; the reference holds no murmur known answers)",
    "cases": [  # key, Long.hashCode, murmurHash, kg(mp=128), operator(p=8)
        [0, 0, 593689054, 94, 5], [1, 1, 68075478, 86, 5], [42, 42, 1134849565, 29, 1],
        [-1, 0, 593689054, 94, 5], [1 << 32, 1, 68075478, 86, 5],
        [-(1 << 63), -2147483648, 1718298732, 108, 6]],
}

# KeyGroupRangeAssignment.computeKeyGroupRangeForOperatorIndex :78-89 — mp=128 over 8 GPUs gives
# [16g, 16g+15]; mp=13 (RescalingITCase.java:133-215 uses mp=13) over p=1..4.
def kg_range(mp, p, i):
    start = 0 if i == 0 else ((i * mp - 1) // p) + 1
    end = ((i + 1) * mp - 1) // p
    return [start, end]


KG_RANGES = {
    "source": "KeyGroupRangeAssignment.java:78-89 (arithmetic transcribed; mp=128,p=8 per SURVEY.md §8e)",
    "cases": [[128, 8, g, 16 * g, 16 * g + 15] for g in range(8)]
             + [[13, p, i] + kg_range(13, p, i) for p in (1, 2, 3, 4) for i in range(p)],
}


def main():
    for fx in FIXTURES:
        with open(os.path.join(HERE, fx["name"] + ".json"), "w") as f:
            json.dump(fx, f, indent=None, separators=(",", ":"))
    with open(os.path.join(HERE, "time_window_start.json"), "w") as f:
        json.dump(WINDOW_START, f, indent=1)
    with open(os.path.join(HERE, "murmur_key_groups.json"), "w") as f:
        json.dump(MURMUR, f, indent=1)
    with open(os.path.join(HERE, "key_group_ranges.json"), "w") as f:
        json.dump(KG_RANGES, f, indent=1)
    print("wrote", len(FIXTURES) + 3, "fixtures to", HERE)


if __name__ == "__main__":
    main()
