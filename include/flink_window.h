/*
 * flink_window.h — C-ABI of the MI355X keyed event-time window aggregation engine.
 *
 * This is the drop-in boundary for Flink's event-time `KeyedStream.window(...).reduce(...)`
 * path, i.e. the non-merging event-time branch of
 *   flink-streaming-java/.../runtime/operators/windowing/WindowOperator.java
 * running on the heap keyed-state backend and the heap timer service.
 *
 * One engine = one operator subtask (one GPU).  A thin JNI shim in a `GpuWindowOperator`
 *  calls these functions; in this repository the Python host mirror
 * (flink_amd/windowing.py) and the tests call them through ctypes.
 *
 * Reference interface each entry point replaces (file:line, paths relative to the reference
 * root, SJ = flink-streaming-java/src/main/java/org/apache/flink/streaming/):
 *
 *   fw_create            <- WindowOperator constructor + open()        SJ/runtime/operators/windowing/WindowOperator.java:150-220
 *                           WindowedStream.reduce -> apply(...)         SJ/api/datastream/WindowedStream.java:185-203,368-425
 *   fw_push_batch        <- WindowOperator.processElement, per record   SJ/runtime/operators/windowing/WindowOperator.java:222-226,302-333
 *                           called by StreamInputProcessor.processInput SJ/runtime/io/StreamInputProcessor.java:169-177
 *                           key groups: KeyGroupRangeAssignment         flink-runtime/.../runtime/state/KeyGroupRangeAssignment.java:51-64
 *   fw_advance_watermark <- AbstractStreamOperator.processWatermark     SJ/api/operators/AbstractStreamOperator.java:803-808
 *                           HeapInternalTimerService.advanceWatermark   SJ/api/operators/HeapInternalTimerService.java:264-278
 *                           WindowOperator.onEventTime                  SJ/runtime/operators/windowing/WindowOperator.java:336-375
 *   fw_collect           <- Output.collect / Output.emitWatermark       SJ/api/operators/Output.java:42-44
 *                           (TimestampedCollector, ts = window.maxTimestamp(): WindowOperator.java:435-438)
 *   fw_get_stats         <- numRecordsIn / numRecordsOut counters       SJ/runtime/io/StreamInputProcessor.java:131-132,173
 *   fw_destroy           <- WindowOperator.close()/dispose()            SJ/api/operators/StreamOperator.java:78,87
 *
 * Conventions
 *  - Every function returns FW_OK (0) or an FW_ERR_* code; no exception crosses the ABI.
 *    fw_last_error() returns a message for the last failure.
 *  - Calls on one engine must be serialised by the caller (mirrors the task checkpoint lock,
 *    SJ/runtime/tasks/StreamTask.java:131).  Engines on different devices are independent.
 *  - fw_push_batch and fw_advance_watermark only ENQUEUE device work; errors found on the device
 *    (Long.MIN_VALUE timestamps, key group outside this subtask's range, capacity) are reported by
 *    the next synchronising call (fw_collect, fw_sync).
 *  - Watermarks: a watermark not larger than the current one changes nothing but still appears as a
 *    mark in the output, as the operator forwards every processWatermark call.
 */
#ifndef FLINK_WINDOW_H
#define FLINK_WINDOW_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- return codes ---- */
#define FW_OK                 0
#define FW_ERR_INVALID_ARG    1  /* bad config / argument                                               */
#define FW_ERR_NO_TIMESTAMP   2  /* record with Long.MIN_VALUE timestamp: TumblingEventTimeWindows.java:60-67 */
#define FW_ERR_CAPACITY       3  /* key directory, slice pool, batch or output log capacity exceeded        */
#define FW_ERR_KEY_GROUP      4  /* key group of a record outside [kg_start, kg_end] of this subtask         */
#define FW_ERR_UNSUPPORTED    5  /* configuration this backend does not implement                            */
#define FW_ERR_DEVICE         6  /* HIP runtime failure                                                      */

/* ---- window assigner (SJ/api/windowing/assigners) ---- */
#define FW_TUMBLING 0            /* TumblingEventTimeWindows.of(size[, offset])  (offset already % size)     */
#define FW_SLIDING  1            /* SlidingEventTimeWindows.of(size, slide[, offset]) (offset already % slide) */
#define FW_SESSION  2            /* EventTimeSessionWindows.withGap(size): merging windows [ts, ts + size)
                                    (SJ/api/windowing/assigners/EventTimeSessionWindows.java:53-56), the merging
                                    branch of WindowOperator.processElement (:228-301) over MergingWindowSet
                                    (SJ/runtime/operators/windowing/MergingWindowSet.java:142-214).  Reduce
                                    fields, first-arrival f1, maxBy / minBy and list state: a merge takes the
                                    merged windows in the JDK HashSet iteration order TimeWindow.mergeWindows
                                    produces (state window = the first one's; the others reduced / their lists
                                    appended in that order), so f1, ties and double sums match the reference.
                                    At most 256 in-flight sessions per key (max_open_slices, default 32:
                                    FW_ERR_CAPACITY beyond).  Reference-layout checkpoints with the
                                    merging-window set (fw_snapshot_kg_flink, reducing state). */

/* ---- trigger (SJ/api/windowing/triggers) ---- */
#define FW_TRIGGER_EVENT_TIME          0   /* EventTimeTrigger.create()                    */
#define FW_TRIGGER_PURGING_EVENT_TIME  1   /* PurgingTrigger.of(EventTimeTrigger.create()) */

/* ---- reduce function: which fields the ReduceFunction aggregates ----
 * The input record is (key, f1, ts, value).  The accumulator is the reduce of the records in
 * arrival order with reduce(value1 = stored, value2 = incoming) (HeapReducingState.java:116):
 *   sum   = value1.sum + value2.sum                (Java long wraps / Java double +)
 *   min   = Math.min(value1.min, value2.min)       (NaN wins, -0.0 < +0.0)
 *   max   = Math.max(value1.max, value2.max)
 *   count = value1.count + value2.count            (each record starts at 1)
 *   f1    = value1.f1                              (first arrival into the pane: SumAggregator.java:64-72)
 * FW_AGG_MAXBY / FW_AGG_MINBY instead return the extremal record (value and f1).
 */
#define FW_AGG_SUM    1
#define FW_AGG_MIN    2
#define FW_AGG_MAX    4
#define FW_AGG_COUNT  8
/* ComparableAggregator MAXBY / MINBY (SJ/api/functions/aggregation/ComparableAggregator.java:66-90,
 * Comparator.java:45-105): the result is the whole extremal record — its value (in the max / min column)
 * and its f1 — ties resolved by FW_AGGF_BY_LAST (first = keep value1, the earlier record).  Used alone. */
#define FW_AGG_MAXBY  16
#define FW_AGG_MINBY  32
/* ListStateDescriptor: WindowedStream.apply(WindowFunction) (WindowedStream.java:244-345) over HeapListState
 * (flink-runtime/.../state/heap/HeapListState.java): the window's elements are buffered (up to list_capacity per
 * pane slice) and a firing window returns every element of every key, grouped by key, in arrival order, one
 * result row per element (value in the sum column, the element's f1, ts = window.maxTimestamp()); the host runs
 * the window function over each group.  Tumbling / sliding: an element arriving for a window that already
 * fired (allowed lateness) re-fires the window for its key with every element so far (under PurgingTrigger:
 * FW_ERR_UNSUPPORTED).  Session windows: each window's elements in list order (a merge appends the sources' lists
 * to the target's, AbstractKeyedStateBackend.mergePartitionedStates :315-333), a late element's per-element fire
 * re-emits the whole list; list_capacity bounds the elements buffered at once (a pool of free entries; entries
 * freed by a batch or watermark are reused from the next one on).  Used alone. */
#define FW_AGG_LIST   64

/* agg_flags */
#define FW_AGGF_COMPARABLE  1  /* min/max order doubles by Double.compareTo (ComparableAggregator .min/.max:
                                  NaN above +inf, -0.0 < +0.0) instead of Math.min/max (NaN wins); long
                                  values order the same either way.  MAXBY/MINBY always use compareTo. */
#define FW_AGGF_BY_LAST     2  /* maxBy/minBy(pos, first = false): a tie takes the later record */
#define FW_AGGF_FOLD        4  /* WindowedStream.fold(initialValue, FoldFunction) (WindowedStream.java:213-242) over
                                  HeapFoldingState (flink-runtime/.../state/heap/HeapFoldingState.java:84-122: the
                                  first add folds into the descriptor's default value): the folds
                                  (acc, v) -> acc + v, acc + 1, Math.min(acc, v), Math.max(acc, v) — one aggregate
                                  (FW_AGG_SUM, FW_AGG_COUNT, FW_AGG_MIN or FW_AGG_MAX) starting from fold_initial
                                  (a long, or a double's bits for a double sum / min / max).  Not with session
                                  windows ("Fold cannot be used with a merging WindowAssigner", :466-467), maxBy /
                                  minBy or first-arrival f1; no checkpoint layout. */

#define FW_VALUE_I64  0
#define FW_VALUE_F64  1

/* memory kinds for buffers crossing the ABI */
#define FW_MEM_HOST    0
#define FW_MEM_DEVICE  1

typedef struct fw_engine fw_engine;

typedef struct {
  int32_t assigner;          /* FW_TUMBLING | FW_SLIDING                                        */
  int32_t trigger;           /* FW_TRIGGER_*                                                    */
  int64_t size;              /* window size (ms)                                                */
  int64_t slide;             /* slide (ms); ignored for tumbling                                */
  int64_t offset;            /* window offset (ms), as held by the assigner                     */
  int64_t allowed_lateness;  /* WindowedStream.allowedLateness (ms), >= 0                       */
  int32_t value_type;        /* FW_VALUE_I64 | FW_VALUE_F64                                     */
  int32_t agg_mask;          /* OR of FW_AGG_*                                                  */
  int32_t keep_first_f1;     /* 1: output f1 of the first arrival into the pane                 */
  int32_t max_parallelism;   /* number of key groups (KeyGroupRangeAssignment, default 128)     */
  int32_t kg_start;          /* first key group owned by this subtask (inclusive)               */
  int32_t kg_end;            /* last key group owned by this subtask (inclusive)                */
  int32_t device;            /* HIP device ordinal                                              */
  int32_t max_open_slices;   /* pane slices resident at once; 0 = derive from the window spec  */
  int64_t key_capacity;      /* distinct keys over the engine lifetime                          */
  int64_t max_batch;         /* max records per fw_push_batch                                   */
  int64_t out_capacity;      /* max fired records between two fw_collect calls                  */
  int32_t ingest_mode;       /* 0 = auto, 1 = direct atomics, 2 = partition + LDS aggregate     */
                             /* (3, the fused form, was removed: FW_ERR_UNSUPPORTED)          */
  int32_t agg_flags;         /* OR of FW_AGGF_*                                                 */
  int64_t fold_initial;      /* FW_AGGF_FOLD: the fold's initial accumulator                    */
  int64_t list_capacity;     /* FW_AGG_LIST: elements buffered per pane slice (session windows: */
                             /* ... in all, live at once); 0 = 4 x max_batch                    */
} fw_config;

/* Output between two collects: records and watermark marks.  Records [mark_pos[i-1], mark_pos[i])
 * are the results emitted before watermark mark_wm[i] was forwarded (records before the first mark
 * have pos 0..mark_pos[0]).  Records after the last mark were emitted by per-element fires that
 * no watermark has followed yet.  Columns that the config does not produce are NULL.
 * Pointers are engine-owned and valid until the next call on the engine. */
typedef struct {
  int64_t n;
  const int64_t* key;
  const int64_t* f1;
  const int64_t* ts;         /* window.maxTimestamp() */
  const int64_t* sum_i64;
  const int64_t* min_i64;
  const int64_t* max_i64;
  const int64_t* count;
  const double*  sum_f64;
  const double*  min_f64;
  const double*  max_f64;
  int64_t n_marks;
  const int64_t* mark_wm;
  const int64_t* mark_pos;
  const int64_t* win_start;  /* FW_SESSION: window.getStart() of each result (window.getEnd() = ts + 1); NULL otherwise */
} fw_out;

typedef struct {
  int64_t records_in;        /* numRecordsIn                                  */
  int64_t records_late;      /* (record, window) pairs dropped by isLate      */
  int64_t panes_fired;       /* timer fires that emitted a result             */
  int64_t late_fires;        /* per-element fires (allowed lateness > 0)      */
  int64_t keys_resident;     /* distinct keys in the key directory            */
  int64_t slices_live;       /* pane slices resident                          */
  int64_t ingest_form;       /* 1 = direct atomics, 2 = partitioned + LDS aggregate */
  int64_t compactions;       /* key-directory compactions (dead keys evicted) */
} fw_stats;

int         fw_create(const fw_config* cfg, fw_engine** out);
/* key: record keys (int64).  key_hash: optional Java key.hashCode() per record (NULL = Long.hashCode(key)).
 * f1: optional pass-through field (NULL = ts).  ts: event timestamps.  value: int64 or double per value_type.
 * mem = FW_MEM_HOST: the call returns once the columns have been copied to the device, so the caller may
 * reuse or release its arrays right away (pageable or pinned alike; e.g. ReleasePrimitiveArrayCritical).
 * mem = FW_MEM_DEVICE: the columns are read asynchronously, after the work enqueued so far on the stream set
 * with fw_set_stream; keep them unchanged until fw_stream_wait_input / fw_sync / fw_collect says they are read. */
int         fw_push_batch(fw_engine* e, const int64_t* key, const int32_t* key_hash, const int64_t* f1,
                          const int64_t* ts, const void* value, int64_t n, int32_t mem);
int         fw_advance_watermark(fw_engine* e, int64_t wm);
int         fw_sync(fw_engine* e);
int         fw_collect(fw_engine* e, fw_out* out, int32_t mem);
/* Asynchronous drain of the same results (the operator hands fired windows downstream while the next batch already
 * runs; they need only precede their watermark, AbstractStreamOperator.java:803-808).  fw_collect_begin enqueues on
 * the engine stream a copy of every result and watermark mark since the last collect into pinned host staging (three
 * buffers, in turn) and restarts the log; it returns at once with a ticket.  fw_collect_end(ticket) waits for
 * that copy and fills `out` (FW_MEM_HOST layout) with columns valid until the next fw_collect_begin after it.  At
 * most three drains are outstanding; one holds at most min(out_capacity, 2^25) results (more: FW_ERR_CAPACITY at
 * fw_collect_end).  Device errors surface at fw_collect_end.  Footprint: each drain's staging is allocated at its
 * first use, sized by capacity, not by results: 3 x (columns x min(out_capacity, 2^25) x 8 B) of
 * pinned host memory plus as much HBM (all 8 columns at out_capacity >= 2^25: 6 GiB pinned + 6 GiB device) —
 * size out_capacity to the results a watermark can fire. */
int         fw_collect_begin(fw_engine* e, int32_t* ticket);
int         fw_collect_end(fw_engine* e, int32_t ticket, fw_out* out);
int         fw_get_stats(fw_engine* e, fw_stats* st);
const char* fw_last_error(const fw_engine* e);
void        fw_destroy(fw_engine* e);

/* ---- checkpoint state per key group ----
 * fw_snapshot_kg <- HeapKeyedStateBackend.snapshot / writeStateTableForKeyGroup
 *                   flink-runtime/.../runtime/state/heap/HeapKeyedStateBackend.java:164-249
 *                   + HeapInternalTimerService.snapshotTimersForKeyGroup   SJ/api/operators/HeapInternalTimerService.java:285-310
 *                   (called per key group from AbstractStreamOperator.snapshotState, AbstractStreamOperator.java:367-391)
 * fw_restore_kg  <- HeapKeyedStateBackend.restorePartitionedState / readStateTableForKeyGroup :251-349
 *                   + HeapInternalTimerService.restoreTimersForKeyGroup :319-345 (AbstractStreamOperator.java:405-425)
 * One blob per key group: FW_SNAP_HEADER_WORDS int64 header words, then n entries of FW_SNAP_ENTRY_WORDS
 * int64 words, native byte order:
 *   header  [0] FW_SNAP_MAGIC  [1] version (2)  [2] key group  [3] n entries  [4] watermark of the snapshot
 *           [5] assigner  [6] size  [7] slide  [8] offset  [9] value_type  [10] agg_mask  [11] keep_first_f1
 *           [12] allowed_lateness  [13] trigger | agg_flags << 8  (words 5-13 must match the restoring engine)
 *   entry   [0] slice number m (namespace: the window [m*size+offset, +size) for tumbling; the slice
 *               [m*g+offset, +g), g = gcd(size, slide), of which every window is made for sliding)
 *           [1] key  [2] sum  [3] min  [4] max  [5] count (double bits / Math.min-max codes for FW_VALUE_F64)
 *           [6] first-arrival order (negative, relative to the end of the snapshot's stream)  [7] f1
 * Timers are implicit, as in the engine: a pane's trigger timer is pending iff its window's maxTimestamp is
 * above the snapshot watermark, its cleanup timer iff it is present at all.  Blobs restored into one engine
 * must carry the same watermark (an aligned checkpoint: every window subtask has seen the same
 * watermarks, which keyBy broadcasts to all of them).  Restore is allowed only before the first push,
 * like initializeState before open.  Keys must be Long keys (no key_hash column was ever pushed).
 * fw_snapshot_kg with buf == NULL (or cap too small) stores the required size in *len and returns
 * FW_OK (NULL) or FW_ERR_CAPACITY. */
#define FW_SNAP_MAGIC         0x31474b5746574bLL   /* "KWFWKG1" */
#define FW_SNAP_HEADER_WORDS  14
#define FW_SNAP_ENTRY_WORDS   8
int         fw_snapshot_kg(fw_engine* e, int32_t kg, void* buf, int64_t cap, int64_t* len);
int         fw_restore_kg(fw_engine* e, int32_t kg, const void* buf, int64_t len);

/* ---- checkpoint state per key group in the reference's own byte layout ----
 * fw_snapshot_kg_flink <- the per-key-group part of HeapKeyedStateBackend.snapshot (HeapKeyedStateBackend.java
 *                         :196-212, writeStateTableForKeyGroup :217-248) and of
 *                         HeapInternalTimerService.snapshotTimersForKeyGroup (:285-310)
 * fw_restore_kg_flink  <- HeapKeyedStateBackend.restorePartitionedState / readStateTableForKeyGroup (:251-349)
 *                         + HeapInternalTimerService.restoreTimersForKeyGroup (:319-345)
 * Two big-endian byte sections per key group, exactly as the JVM writes them:
 *   state   the bytes at KeyGroupRangeOffsets[kg] of the managed keyed-state stream:
 *             int kg | short 0 (id of "window-contents", the operator's only keyed state) | byte present |
 *             [int numNamespaces | (long start | long end | int n | (long key | state tuple) * n) * numNamespaces]
 *           present = the key group ever held window state (StateTable.get(kg) != null).
 *   timers  the body of snapshotTimersForKeyGroup after its two InstantiationUtil.serializeObject records:
 *             int n | (long key | long start | long end | long timestamp) * n | int 0 (processing-time timers)
 *           The caller writes the raw keyed-state prologue around it (AbstractStreamOperator.snapshotState
 *           :367-391: int 1, writeUTF("window-timers"), the Java-serialized key and namespace serializers):
 *           JVM object serialization stays on the JVM side.
 * The state tuple is the ReduceFunction's value type: layout->field[0..n_fields) in tuple order, each an
 * 8-byte LongSerializer / DoubleSerializer field (TupleSerializer.serialize :120-129).  The layout must
 * name every aggregate the config computes (FW_SF_VALUE for maxBy/minBy), FW_SF_F1 iff keep_first_f1,
 * FW_SF_KEY at most once.  Fold (FW_AGGF_FOLD): the state is HeapFoldingState's accumulator, the initial value
 * folded with the pane (the layout names the one aggregate).  List state (FW_AGG_LIST):
 * the state is ListSerializer's `int size | element * size`, each element the window's input tuple with the
 * fields the layout names — FW_SF_VALUE once, FW_SF_KEY and FW_SF_F1 at most once each — in arrival order.
 * Session windows (reducing state): two tables, ids in stateTables' HashMap order (WindowOperator.java:445-460,
 * 724-736): short 0 "window-contents" as above, its namespaces the in-flight windows' STATE windows (a session's
 * first window [ts, ts + gap): MergingWindowSet keeps the first merged window's state window), then short 1
 * "merging-window-set" | byte present | [int 0 or 1 | byte 0 (VoidNamespace) | int n | (long key | int m |
 * (long start | long end | long stateStart | long stateEnd) * m) * n] (ListState<Tuple2<W, W>>,
 * MergingWindowSet.persist :91-95) as WindowOperator.snapshotState rewrites it: restored entries of keys untouched
 * since, then every other key with sessions in flight in mergingWindowsByKey's order.  Timers: each in-flight
 * window's pending trigger timer and its cleanup timer (PurgingTrigger with allowed lateness: also purged
 * sessions' cleanup timers until their time); list state: each window's elements in list order.
 * Namespaces, entries and timers come in java.util.HashMap iteration order for
 * tables sized by their current size (when a JVM table iterates differently).
 * A buffer argument NULL (or too small: FW_ERR_CAPACITY) stores the required lengths only.
 * *state_len == 0: no keyed state at all yet (no record accepted, nothing restored), for which
 * HeapKeyedStateBackend.snapshot writes no stream (:169-171).
 * Restore: before the first push.  Tumbling windows restore into their slices; sliding windows into each
 * window's own pane (later records go to slices; a window fires its slices and its pane); sliding list state
 * into the slices, peeled from the windows' lists.  PurgingTrigger with allowed lateness > 0: a purged window's
 * keys keep their cleanup timers without state (tumbling: ghost ordinals per slice slot; sliding: restored as
 * such, and derived at snapshot for windows fired since — keys whose first element preceded the fire, which needs
 * keep_first_f1).
 * `watermark` is the engine's watermark after restore: the reference restarts its timer service at
 * Long.MIN_VALUE (currentWatermark is not checkpointed) — pass INT64_MIN for exactly that.  The engine's
 * timers are implicit (a pane's trigger timer is pending iff its window's maxTimestamp > watermark, its
 * cleanup timer iff the pane exists), so the blob's timers must be the ones its panes imply at `watermark`,
 * with one exception the reference's own checkpoints produce: a tumbling window ahead of `watermark` whose
 * panes carry no trigger timer (it fired before the checkpoint and is kept for its allowed lateness) is
 * restored disarmed — it fires again only for keys whose records re-arm it before the watermark passes its
 * maxTimestamp (EventTimeTrigger.onElement), otherwise it waits for its cleanup time; a sliding window likewise,
 * through its own pane, and tumbling list state through its slice.  Every restored key
 * group must use the same `watermark`. */
#define FW_SF_KEY    1   /* the key (the tuple's key field, e.g. f0)                          */
#define FW_SF_F1     2   /* the pass-through field of the first arrival (maxBy/minBy: of the extremal record) */
#define FW_SF_SUM    3
#define FW_SF_MIN    4
#define FW_SF_MAX    5
#define FW_SF_COUNT  6   /* long                                                              */
#define FW_SF_VALUE  7   /* maxBy/minBy: the extremal record's value field                    */
#define FW_SF_MAX_FIELDS 8
typedef struct {
  int32_t n_fields;
  int32_t field[FW_SF_MAX_FIELDS];
} fw_state_layout;
int         fw_snapshot_kg_flink(fw_engine* e, int32_t kg, const fw_state_layout* layout, void* state,
                                 int64_t state_cap, int64_t* state_len, void* timers, int64_t timers_cap,
                                 int64_t* timers_len);
int         fw_restore_kg_flink(fw_engine* e, int32_t kg, const fw_state_layout* layout, int64_t watermark,
                                const void* state, int64_t state_len, const void* timers, int64_t timers_len);

/* ---- ingest from Flink's wire format ----
 * fw_decode <- the receiving side of a channel: SpillingAdaptiveSpanningRecordDeserializer reassembling
 *              length-prefixed records from network buffers (written by SpanningRecordSerializer.addRecord,
 *              flink-runtime/.../io/network/api/serialization/SpanningRecordSerializer.java:69-92: int32 BE
 *              length, then the bytes) + StreamElementSerializer.deserialize
 *              (SJ/runtime/streamrecord/StreamElementSerializer.java:155-198: tag byte 0 record with
 *              timestamp (int64 BE follows), 1 record without, 2 watermark (int64), 3 latency marker
 *              (int64, int32, int32)) + TupleSerializer.deserialize (flink-core/.../typeutils/runtime/
 *              TupleSerializer.java:120-139: the fields in order, LongSerializer / DoubleSerializer /
 *              IntSerializer big-endian), as StreamInputProcessor.processInput drives them (:127-177).
 * `bytes` is the concatenation of the buffers' contents (nbytes, FW_MEM_HOST or FW_MEM_DEVICE) starting at
 * an element boundary; an element cut by the end stays for the next call (*consumed < nbytes: pass the
 * rest again in front of the next buffers).  Records are decoded, on the GPU, into device columns ready
 * for fw_push_batch(FW_MEM_DEVICE): key, key_hash (an int key's Integer.hashCode; NULL for long keys),
 * f1 (the schema's f1 field, or the timestamp), ts (Long.MIN_VALUE for a record without timestamp) and
 * value (long or double bits).  Watermarks and latency markers come back in stream order with their
 * position: the number of records before them (device arrays).  A malformed stream (no element chain
 * through the bytes) fails with FW_ERR_INVALID_ARG. */
#define FW_FT_LONG    0   /* LongSerializer: 8 bytes                              */
#define FW_FT_DOUBLE  1   /* DoubleSerializer: 8 bytes (the value field only)     */
#define FW_FT_INT     2   /* IntSerializer: 4 bytes (key or f1; sign-extended)    */
#define FW_DECODE_MAX_FIELDS 8
typedef struct {
  int32_t n_fields;                        /* the tuple's arity                            */
  int32_t field_type[FW_DECODE_MAX_FIELDS];
  int32_t key_field;                       /* index of the key field                        */
  int32_t f1_field;                        /* index of the pass-through field, -1: the ts   */
  int32_t value_field;                     /* index of the reduced field                    */
} fw_tuple_schema;
typedef struct {
  int64_t n_records, n_watermarks, n_latency_markers;
  int64_t consumed;                        /* bytes of whole elements decoded               */
} fw_decode_counts;
int         fw_decode(fw_engine* e, const fw_tuple_schema* schema, const void* bytes, int64_t nbytes, int32_t mem,
                      int64_t* key, int32_t* key_hash, int64_t* f1, int64_t* ts, void* value, int64_t record_cap,
                      int64_t* wm, int64_t* wm_pos, int64_t* lm, int64_t* lm_pos, int64_t marker_cap,
                      fw_decode_counts* out);
/* The same in two halves, so the count read-back of one buffer overlaps the next buffer's kernels:
 * fw_decode_begin enqueues the decode on the engine stream and returns a ticket at once; fw_decode_end(ticket)
 * waits for it and reports its counts (the errors fw_decode reports surface there).  At most two decodes are
 * outstanding; a host input (FW_MEM_HOST) and the output columns must stay untouched until fw_decode_end. */
int         fw_decode_begin(fw_engine* e, const fw_tuple_schema* schema, const void* bytes, int64_t nbytes, int32_t mem,
                            int64_t* key, int32_t* key_hash, int64_t* f1, int64_t* ts, void* value, int64_t record_cap,
                            int64_t* wm, int64_t* wm_pos, int64_t* lm, int64_t* lm_pos, int64_t marker_cap,
                            int32_t* ticket);
int         fw_decode_end(fw_engine* e, int32_t ticket, fw_decode_counts* out);

/* Key-group routing for the multi-GPU keyBy exchange (enqueued on the caller stream when fw_set_stream set one)
 * (KeyGroupStreamPartitioner.selectChannels, SJ/runtime/partitioner/KeyGroupStreamPartitioner.java:52-65;
 *  KeyGroupRangeAssignment.assignKeyToParallelOperator, KeyGroupRangeAssignment.java:40-42,105-107).
 * Counting-sorts n records by destination operator index into out_* (device pointers) and writes
 * per-destination counts and offsets (int64[parallelism]).  Stable within a destination. */
int         fw_partition_by_operator(fw_engine* e, const int64_t* key, const int32_t* key_hash,
                                     const int64_t* f1, const int64_t* ts, const void* value, int64_t n,
                                     int32_t max_parallelism, int32_t parallelism,
                                     int64_t* out_key, int32_t* out_key_hash, int64_t* out_f1,
                                     int64_t* out_ts, void* out_value, int64_t* counts, int64_t* offsets);
/* The same with operator `last_operator`'s records placed after every other operator's (output order
 * last+1 .. parallelism-1, 0 .. last; counts stay indexed by operator, offsets[d] is operator d's start): a
 * receiving subtask lands its peers' records right behind its own share in the same columns and pushes the
 * whole in one fw_push_batch.  last_operator < 0: operator order, as fw_partition_by_operator. */
int         fw_partition_by_operator_last(fw_engine* e, const int64_t* key, const int32_t* key_hash,
                                          const int64_t* f1, const int64_t* ts, const void* value, int64_t n,
                                          int32_t max_parallelism, int32_t parallelism,
                                          int64_t* out_key, int32_t* out_key_hash, int64_t* out_f1,
                                          int64_t* out_ts, void* out_value, int64_t* counts, int64_t* offsets,
                                          int32_t last_operator);

/* Device-time accounting (HIP events around each kernel, on the stream it runs on), for the roofline
 * figures of bench.py.  Off by default; enabling it adds timed event records between kernels, which
 * serialise them (measure throughput with it off). */
#define FW_PHASE_INGEST  0   /* per-record ingest: k_route (partitioned form) or k_ingest_direct */
#define FW_PHASE_FIXUP   1   /* first-arrival f1 gather for new panes (direct form)           */
#define FW_PHASE_LATE    2   /* per-element fires (allowed lateness > 0)                      */
#define FW_PHASE_FIRE    3   /* watermark: plan + fire + purge + mark (k_watermark)            */
#define FW_PHASE_AGGREGATE 4 /* partitioned form: per-bucket LDS aggregation (k_aggregate)    */
#define FW_NPHASES       5
typedef struct {
  double  ms[FW_NPHASES];        /* accumulated device milliseconds per phase */
  int64_t launches[FW_NPHASES];  /* timed launches per phase                  */
  int64_t records[FW_NPHASES];   /* records (ingest) or panes scanned (fire)  */
} fw_profile;
int         fw_set_profiling(fw_engine* e, int32_t enable);
int         fw_get_profile(fw_engine* e, fw_profile* out);   /* synchronises; resets the counters */

/* Make the caller's HIP stream (hipStream_t; 0 = the null stream) the producer of device-resident input
 * columns: every push waits for the work enqueued on it so far, and fw_partition_by_operator runs on it.
 * Synchronises first. */
int         fw_set_stream(fw_engine* e, void* stream);
/* Make `stream` wait (device-side, no host synchronisation) until the engine has finished reading the
 * input columns of the non-empty push made `back` pushes ago (0 = the latest, at most 7), so that a caller
 * recycling column buffers never overwrites one the engine still reads. */
int         fw_stream_wait_input(fw_engine* e, void* stream, int32_t back);

/* diagnostics: raw device counters (8 x int64) */
int         fw_debug_counters(fw_engine* e, int64_t* out8);
/* diagnostics: per-workgroup phase timestamps of the partitioned ingest (engine created with
 * FW_DEBUG_AGG & 16 in the environment); n int64 values, 100 MHz realtime clock */
int         fw_debug_stamps(fw_engine* e, int64_t* out, int64_t n);

/* library version string */
const char* fw_version(void);

#ifdef __cplusplus
}
#endif
#endif
