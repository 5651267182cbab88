// fw_list.hip — list window state on the GPU (included by fw_engine.hip).
//
// Replaces HeapListState under WindowedStream.apply(WindowFunction) (WindowedStream.java:244-345; the
// operator's ListStateDescriptor "window-contents"): every element of a window is kept, and a firing
// window hands the window function all of them (InternalIterableWindowFunction) in arrival order
// (HeapListState.add appends; its Iterable iterates in insertion order).
//
// Layout: the pane slices of the reduce path (a record belongs to exactly one slice however many sliding
// windows cover it), each with a buffer of elements (kid, arrival ordinal, value, f1).  A firing window
// gathers its K slices' elements, sorts them by arrival ordinal and then (stably) by key id — rocPRIM
// radix sorts — and appends one result row per element, grouped by key, to the output log; the host
// runs the window function over each (key, window) group.  A slice is dropped when its last window's
// cleanup time passes, like the reduce path's purge.  An element for a window that already fired but is
// not yet cleaned up (allowed lateness) is added and re-fires the window for its key with every element so
// far (EventTimeTrigger.onElement FIRE, WindowOperator.java:302-333): each such (key, window, arrival) is
// listed at ingest; after the batch the window's elements are gathered and sorted as for a watermark fire,
// and each listed fire emits its key's elements up to its own arrival.  PurgingTrigger with such fires
// (the purge would clear one window of slices other windows share) stays FW_ERR_UNSUPPORTED.

namespace fw {

// k_list_plan output: [0] windows firing, [1] slots purged, then WM_MAXT (window, elements) pairs, then
// WM_MAXP purged slots
constexpr int LPLAN_WORDS = 2 + 2 * WM_MAXT + WM_MAXP;

__global__ __launch_bounds__(BLOCK) void k_list_ingest(Spec s, BatchIn b, ListDev L) {
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x; i0 < b.n; i0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = i0 + threadIdx.x;   // uniform loop: every lane takes part in the wave appends
    bool live = false;
    int32_t p = -1;
    int64_t kid = -1, ts = 0;
    unsigned long long late = 0;
    if (i < b.n) {
      const int64_t key = b.key[i];
      ts = b.ts[i];
      const int32_t h = b.key_hash ? b.key_hash[i] : long_hash_code(key);
      bool ok = true;
      if (ts == INT64_MIN) { set_error(s.err, FW_ERR_NO_TIMESTAMP); ok = false; }
      const int32_t kg = record_key_group(s, h);
      if (ok && (kg < s.kg_start || kg > s.kg_end)) { set_error(s.err, FW_ERR_KEY_GROUP); ok = false; }
      if (ok) {
        const RecWin w = record_windows(s, ts, b.wm);
        late = (unsigned long long)w.n_late + (w.q_late ? 1ull : 0ull);
        if ((w.n_fire > 0 && s.trigger == FW_TRIGGER_PURGING_EVENT_TIME) || (w.quirk && !w.q_late)) {
          set_error(s.err, FW_ERR_UNSUPPORTED);
          ok = false;
        }
        live = ok && (w.n_windows - w.n_late) > 0;
        if (live) {
          p = slice_slot(s, w.m);
          kid = dir_find_or_insert(s, key);
          if (p < 0 || kid < 0) { cap_error(s, 24); live = false; }
        }
        if (live && w.n_fire > 0) {   // the windows of the record that fired already: one re-fire each
          for (int64_t n = floor_div(w.m - s.K, s.R) + 1; n <= floor_div(w.m, s.R); ++n) {
            const int64_t max_ts = jsub(jadd(window_start_n(s, n), s.size), 1);
            if (max_ts > b.wm || cleanup_time(max_ts, s.lateness) <= b.wm) continue;
            const unsigned long long f = atomicAdd(L.fcnt, 1ull);
            if ((int64_t)f >= L.fcap) { cap_error(s, 27); continue; }
            L.fire[3 * f] = kid;
            L.fire[3 * f + 1] = n;
            L.fire[3 * f + 2] = b.ord_base + i;
          }
        }
      }
    }
    if (__any(late != 0)) {
      for (int o = 32; o > 0; o >>= 1) late += __shfl_xor(late, o);
      if ((threadIdx.x & 63) == 0 && late) atomicAdd(&s.stats[ST_LATE], late);
    }
    // wave-aggregated append when the wave's live records share one slice (an in-order stream)
    const uint64_t lm = __ballot(live);
    if (lm == 0) continue;
    const int leader = __ffsll((long long)lm) - 1;
    const int32_t p0 = __shfl(p, leader);
    unsigned long long pos;
    if (__all(!live || p == p0)) pos = wave_append(&L.cnt[p0], live);
    else pos = live ? atomicAdd(&L.cnt[p], 1ull) : 0;
    if (!live) continue;
    if ((int64_t)pos >= L.cap) { cap_error(s, 25); continue; }
    int64_t* el = L.buf + ((int64_t)p * L.cap + (int64_t)pos) * LST_WORDS;
    el[0] = kid;
    el[1] = b.ord_base + i;
    el[2] = b.val[i];
    el[3] = b.f1 ? b.f1[i] : ts;
  }
}

// the firing windows (maxTimestamp in (old, new], a live slice) with their element counts, and the slices
// whose last window's cleanup time passed
__global__ __launch_bounds__(1024) void k_list_plan(Spec s, ListDev L, int64_t wm_old, int64_t wm_new, int64_t* plan) {
  __shared__ int32_t nt, np;
  if (threadIdx.x == 0) { nt = 0; np = 0; }
  __syncthreads();
  for (int32_t p = threadIdx.x; p < s.P; p += blockDim.x) {
    const int64_t m = s.slice_tag[p];
    if (m == FREE_TAG) continue;
    const int64_t n_hi = floor_div(m, s.R), n_lo = floor_div(m - s.K, s.R) + 1;
    for (int64_t n = n_lo; n <= n_hi; ++n) {
      const int64_t max_ts = jsub(jadd(window_start_n(s, n), s.size), 1);
      if (!(max_ts > wm_old && max_ts <= wm_new)) continue;
      bool owner = true;   // the first live slice of window n lists it
      for (int64_t mm = n * s.R; mm < m; ++mm)
        if (s.slice_tag[floor_mod(mm, s.P)] == mm) { owner = false; break; }
      if (!owner) continue;
      int64_t cnt = 0;
      for (int64_t mm = n * s.R; mm < n * s.R + s.K; ++mm) {
        const int32_t pp = (int32_t)floor_mod(mm, s.P);
        if (s.slice_tag[pp] == mm) cnt += (int64_t)min((unsigned long long)L.cap, L.cnt[pp]);
      }
      const int32_t t = atomicAdd(&nt, 1);
      if (t < WM_MAXT) { plan[2 + 2 * t] = n; plan[3 + 2 * t] = cnt; }
      else cap_error(s, 26);
    }
    const int64_t ct = cleanup_time(jsub(jadd(window_start_n(s, n_hi), s.size), 1), s.lateness);
    if (ct <= wm_new) {
      const int32_t q = atomicAdd(&np, 1);
      if (q < WM_MAXP) plan[2 + 2 * WM_MAXT + q] = p;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) { plan[0] = min(nt, WM_MAXT); plan[1] = min(np, WM_MAXP); }
}

// window n's elements: sort keys (arrival ordinal) and their buffer positions
__global__ __launch_bounds__(BLOCK) void k_list_gather(Spec s, ListDev L, int64_t n, unsigned long long* key, int64_t* idx) {
  int64_t off[LIST_MAX_K + 1];
  int32_t slot[LIST_MAX_K];
  off[0] = 0;
  for (int k = 0; k < s.K; ++k) {
    const int64_t mm = n * s.R + k;
    const int32_t pp = (int32_t)floor_mod(mm, s.P);
    const bool live = s.slice_tag[pp] == mm;
    slot[k] = pp;
    off[k + 1] = off[k] + (live ? (int64_t)min((unsigned long long)L.cap, L.cnt[pp]) : 0);
  }
  const int64_t total = off[s.K];
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    int k = 0;
    while (off[k + 1] <= e) ++k;
    const int64_t at = ((int64_t)slot[k] * L.cap + (e - off[k])) * LST_WORDS;
    key[e] = (unsigned long long)L.buf[at + 1] ^ 0x8000000000000000ull;   // ordinal, order-preserving unsigned
    idx[e] = at;
  }
}

__global__ __launch_bounds__(BLOCK) void k_list_kid(ListDev L, const int64_t* idx, int64_t N, unsigned long long* key) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < N; e += (int64_t)gridDim.x * blockDim.x)
    key[e] = (unsigned long long)L.buf[idx[e]];
}

// one result row per element, grouped by key (sorted), at output positions base..base+N
__global__ __launch_bounds__(BLOCK) void k_list_emit(Spec s, ListDev L, const int64_t* idx, int64_t N, int64_t base,
                                                     int64_t max_ts) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < N; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t* el = L.buf + idx[e];
    const int64_t pos = base + e;
    const bool head = e == 0 || L.buf[idx[e - 1]] != el[0];
    wave_count(&s.stats[ST_FIRED], head);   // one fire per (key, window)
    if (pos >= s.o.capacity) { cap_error(s, 11); continue; }
    s.o.key[pos] = kid_key(s, el[0]);
    s.o.f1[pos] = el[3];
    s.o.ts[pos] = max_ts;
    s.o.sum[pos] = el[2];
  }
}

// per-element re-fires of window n (pairs (kid, arrival ordinal) in arrival order): the element count of
// each — its key's elements of the window (sorted by key id, then arrival: kids[], pos[]) up to its arrival
__global__ __launch_bounds__(BLOCK) void k_list_fire_count(ListDev L, const unsigned long long* kids, const int64_t* pos,
                                                          int64_t N, const int64_t* pairs, int64_t F, int64_t* cnt) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < F; j += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long kid = (unsigned long long)pairs[2 * j];
    const int64_t ord = pairs[2 * j + 1];
    int64_t lo = 0, hi = N;   // first element of the key
    while (lo < hi) { const int64_t mid = (lo + hi) >> 1; if (kids[mid] < kid) lo = mid + 1; else hi = mid; }
    int64_t a = lo, z = N;    // first element of the key after its arrival (ordinals increase within a key)
    while (a < z) {
      const int64_t mid = (a + z) >> 1;
      if (kids[mid] == kid && L.buf[pos[mid] + 1] <= ord) a = mid + 1; else z = mid;
    }
    cnt[2 * j] = lo;
    cnt[2 * j + 1] = a - lo;
  }
}

// their rows at base + off[j]: the window's elements of the key, in arrival order (ts = window.maxTimestamp())
__global__ __launch_bounds__(BLOCK) void k_list_fire_emit(Spec s, ListDev L, const int64_t* pos, const int64_t* cnt,
                                                         const int64_t* off, int64_t F, int64_t base, int64_t max_ts) {
  for (int64_t j = blockIdx.x; j < F; j += gridDim.x) {
    const int64_t lo = cnt[2 * j], c = cnt[2 * j + 1];
    for (int64_t e = threadIdx.x; e < c; e += blockDim.x) {
      const int64_t* el = L.buf + pos[lo + e];
      const int64_t at = base + off[j] + e;
      if (at >= s.o.capacity) { cap_error(s, 11); continue; }
      s.o.key[at] = kid_key(s, el[0]);
      s.o.f1[at] = el[3];
      s.o.ts[at] = max_ts;
      s.o.sum[at] = el[2];
    }
  }
}

__global__ void k_list_set_count(Spec s, int64_t count) { *s.o.count = (unsigned long long)count; }

// output count; the expired slices' buffers and slots freed
__global__ void k_list_finish(Spec s, ListDev L, const int64_t* plan, int64_t count) {
  const int64_t np = plan[1];
  for (int64_t q = threadIdx.x; q < np; q += blockDim.x) {
    const int32_t p = (int32_t)plan[2 + 2 * WM_MAXT + q];
    L.cnt[p] = 0;
    s.slice_tag[p] = FREE_TAG;
  }
  if (threadIdx.x == 0) *s.o.count = (unsigned long long)count;
}

}  // namespace fw

using namespace fw;

int list_create(fw_engine* e) {
  const Spec& s = e->s;
  ListDev& L = e->lst;
  L.cap = e->cfg.list_capacity > 0 ? e->cfg.list_capacity : 4 * e->cfg.max_batch;
  L.cnt = e->alloc<unsigned long long>((size_t)s.P);
  L.buf = e->alloc<int64_t>((size_t)s.P * (size_t)L.cap * LST_WORDS);
  if (e->cfg.allowed_lateness > 0) {   // per-element re-fires: (kid, window, arrival) of one batch
    L.fcap = e->cfg.max_batch * (int64_t)((s.K + s.R - 1) / s.R);   // a record re-fires each of its windows
    L.fire = e->alloc<int64_t>((size_t)L.fcap * 3);
    L.fcnt = e->alloc<unsigned long long>(1);
  }
  e->list_plan = e->alloc<int64_t>(LPLAN_WORDS);
  e->list_plan_h.resize(LPLAN_WORDS);
  for (void* p : e->allocs) if (!p) return FW_ERR_DEVICE;
  HIPCHK(e, hipMemsetAsync(L.cnt, 0, 8 * (size_t)s.P, e->stream));
  if (L.fcnt) HIPCHK(e, hipMemsetAsync(L.fcnt, 0, 8, e->stream));
  return FW_OK;
}

static int list_grow(fw_engine* e, int64_t n);
static int list_sort_window(fw_engine* e, int64_t n, int64_t N);

int list_push(fw_engine* e, const BatchIn& b) {
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((b.n + BLOCK - 1) / BLOCK, e->grid));
  e->phase_begin(FW_PHASE_INGEST);
  DBGSYNC(e, "push entry");
  hipLaunchKernelGGL(k_list_ingest, dim3(blocks), dim3(BLOCK), 0, e->stream, e->s, b, e->lst);
  DBGSYNC(e, "k_list_ingest");
  e->phase_end(b.n);
  HIPCHK(e, hipGetLastError());
  if (!e->lst.fcnt || !fires_possible(e->s, e->cur_wm)) return FW_OK;
  // per-element re-fires (allowed lateness): the batch's list, grouped by window in arrival order
  unsigned long long F = 0;
  HIPCHK(e, hipMemcpyAsync(&F, e->lst.fcnt, 8, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  F = std::min<unsigned long long>(F, (unsigned long long)e->lst.fcap);
  if (F == 0) return FW_OK;
  std::vector<int64_t> fl(3 * F);
  HIPCHK(e, hipMemcpy(fl.data(), e->lst.fire, 8 * 3 * F, hipMemcpyDeviceToHost));
  HIPCHK(e, hipMemsetAsync(e->lst.fcnt, 0, 8, e->stream));
  std::map<int64_t, std::vector<std::pair<int64_t, int64_t>>> by_win;   // window -> (arrival, kid)
  for (unsigned long long j = 0; j < F; ++j) by_win[fl[3 * j + 1]].push_back({fl[3 * j + 2], fl[3 * j]});
  e->phase_begin(FW_PHASE_LATE);
  for (auto& wv : by_win) {
    const int64_t n = wv.first;
    auto& pr = wv.second;
    std::sort(pr.begin(), pr.end());
    // the window's elements, sorted by key id then arrival (its count from the live slices' counters)
    std::vector<unsigned long long> cnts((size_t)e->s.P);
    std::vector<int64_t> tags((size_t)e->s.P);
    HIPCHK(e, hipMemcpy(cnts.data(), e->lst.cnt, 8 * (size_t)e->s.P, hipMemcpyDeviceToHost));
    HIPCHK(e, hipMemcpy(tags.data(), e->s.slice_tag, 8 * (size_t)e->s.P, hipMemcpyDeviceToHost));
    int64_t N = 0;
    for (int64_t mm = n * e->s.R; mm < n * e->s.R + e->s.K; ++mm) {
      const int32_t pp = (int32_t)floor_mod(mm, e->s.P);
      if (tags[(size_t)pp] == mm) N += (int64_t)std::min<unsigned long long>((unsigned long long)e->lst.cap, cnts[(size_t)pp]);
    }
    if (N == 0) continue;
    if (int rc = list_sort_window(e, n, N)) return rc;   // kids in list_k2, positions in list_v1
    const int64_t Fn = (int64_t)pr.size();
    std::vector<int64_t> pairs(2 * (size_t)Fn), cnt(2 * (size_t)Fn), off((size_t)Fn);
    for (int64_t j = 0; j < Fn; ++j) { pairs[2 * (size_t)j] = pr[(size_t)j].second; pairs[2 * (size_t)j + 1] = pr[(size_t)j].first; }
    if (5 * Fn > e->list_fire_cap) {   // grow-only scratch (pairs, counts, offsets), freed with the engine
      HIPCHK(e, hipStreamSynchronize(e->stream));
      if (e->list_fire_dp) (void)hipFree(e->list_fire_dp);
      e->list_fire_dp = nullptr;
      e->list_fire_cap = 0;
      HIPCHK(e, hipMalloc((void**)&e->list_fire_dp, 8 * (size_t)(10 * Fn)));
      e->list_fire_cap = 10 * Fn;
    }
    int64_t* dp = e->list_fire_dp;
    HIPCHK(e, hipMemcpy(dp, pairs.data(), 16 * (size_t)Fn, hipMemcpyHostToDevice));
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((Fn + BLOCK - 1) / BLOCK, e->grid));
    hipLaunchKernelGGL(k_list_fire_count, dim3(blocks), dim3(BLOCK), 0, e->stream, e->lst, e->list_k2, e->list_v1, N, dp,
                       Fn, dp + 2 * Fn);
    DBGSYNC(e, "k_list_fire_count");
    HIPCHK(e, hipMemcpyAsync(cnt.data(), dp + 2 * Fn, 16 * (size_t)Fn, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    int64_t tot = 0;
    for (int64_t j = 0; j < Fn; ++j) { off[(size_t)j] = tot; tot += cnt[2 * (size_t)j + 1]; }
    if (e->list_out + tot > e->cfg.out_capacity) return fail(e, FW_ERR_CAPACITY, "output log capacity exceeded (list state)");
    HIPCHK(e, hipMemcpy(dp + 4 * Fn, off.data(), 8 * (size_t)Fn, hipMemcpyHostToDevice));
    const int64_t max_ts = jsub(jadd(jadd(e->s.offset, (int64_t)((uint64_t)n * (uint64_t)e->s.slide)), e->s.size), 1);
    hipLaunchKernelGGL(k_list_fire_emit, dim3((unsigned)std::min<int64_t>(Fn, 4096)), dim3(BLOCK), 0, e->stream, e->s,
                       e->lst, e->list_v1, dp + 2 * Fn, dp + 4 * Fn, Fn, e->list_out, max_ts);
    DBGSYNC(e, "k_list_fire_emit");
    HIPCHK(e, hipStreamSynchronize(e->stream));
    e->list_out += tot;
    e->late_fires_host += Fn;
  }
  hipLaunchKernelGGL(k_list_set_count, dim3(1), dim3(1), 0, e->stream, e->s, e->list_out);
  e->phase_end((int64_t)F);
  HIPCHK(e, hipGetLastError());
  e->out_dirty = true;
  return FW_OK;
}

static int list_grow(fw_engine* e, int64_t n) {
  if (n <= e->list_tmp_cap) return FW_OK;
  HIPCHK(e, hipStreamSynchronize(e->stream));
  for (void* p : {(void*)e->list_k1, (void*)e->list_k2, (void*)e->list_v1, (void*)e->list_v2, e->list_temp})
    if (p) (void)hipFree(p);
  const int64_t cap = std::max<int64_t>(n, 2 * e->list_tmp_cap);
  HIPCHK(e, hipMalloc((void**)&e->list_k1, 8 * (size_t)cap));
  HIPCHK(e, hipMalloc((void**)&e->list_k2, 8 * (size_t)cap));
  HIPCHK(e, hipMalloc((void**)&e->list_v1, 8 * (size_t)cap));
  HIPCHK(e, hipMalloc((void**)&e->list_v2, 8 * (size_t)cap));
  size_t tb = 0;
  HIPCHK(e, rocprim::radix_sort_pairs(nullptr, tb, e->list_k1, e->list_k2, e->list_v1, e->list_v2, (size_t)cap, 0, 64,
                                      e->stream));
  e->list_temp_bytes = tb;
  HIPCHK(e, hipMalloc(&e->list_temp, tb));
  e->list_tmp_cap = cap;
  return FW_OK;
}

// window n's N elements gathered and sorted: arrival order, then (stably) grouped by key id — the sorted key
// ids in list_k2, the elements' buffer positions in list_v1
static int list_sort_window(fw_engine* e, int64_t n, int64_t N) {
  if (int rc = list_grow(e, N)) return rc;
  const int kid_bits = bits_for((uint64_t)e->s.stride);
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((N + BLOCK - 1) / BLOCK, e->grid));
  hipLaunchKernelGGL(k_list_gather, dim3(blocks), dim3(BLOCK), 0, e->stream, e->s, e->lst, n, e->list_k1, e->list_v1);
  DBGSYNC(e, "k_list_gather");
  size_t tb = e->list_temp_bytes;
  HIPCHK(e, rocprim::radix_sort_pairs(e->list_temp, tb, e->list_k1, e->list_k2, e->list_v1, e->list_v2, (size_t)N, 0, 64,
                                      e->stream));
  DBGSYNC(e, "radix sort 1");
  hipLaunchKernelGGL(k_list_kid, dim3(blocks), dim3(BLOCK), 0, e->stream, e->lst, e->list_v2, N, e->list_k1);
  DBGSYNC(e, "k_list_kid");
  tb = e->list_temp_bytes;
  HIPCHK(e, rocprim::radix_sort_pairs(e->list_temp, tb, e->list_k1, e->list_k2, e->list_v2, e->list_v1, (size_t)N, 0,
                                      kid_bits, e->stream));
  DBGSYNC(e, "radix sort 2");
  return FW_OK;
}

int list_watermark(fw_engine* e, int64_t wm) {
  if (wm <= e->cur_wm || wm_quiet(e->s, e->cur_wm, wm)) {   // nothing fires or purges: the mark only
    if (e->out_dirty) {   // per-element re-fires appended since the last device mark
      hipLaunchKernelGGL(k_mark_only, dim3(1), dim3(1), 0, e->stream, e->s, wm);
      HIPCHK(e, hipGetLastError());
      e->hmarks.push_back({wm, e->dev_marks++, true});
      e->out_dirty = false;
    } else {
      e->hmarks.push_back({wm, e->dev_marks - 1, false});
    }
    if (wm > e->cur_wm) e->cur_wm = wm;
    return FW_OK;
  }
  e->phase_begin(FW_PHASE_FIRE);
  DBGSYNC(e, "watermark entry");
  hipLaunchKernelGGL(k_list_plan, dim3(1), dim3(1024), 0, e->stream, e->s, e->lst, e->cur_wm, wm, e->list_plan);
  DBGSYNC(e, "k_list_plan");
  HIPCHK(e, hipMemcpyAsync(e->list_plan_h.data(), e->list_plan, 8 * LPLAN_WORDS, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(e, hipStreamSynchronize(e->stream));
  const int64_t nt = e->list_plan_h[0];
  for (int64_t t = 0; t < nt; ++t) {
    const int64_t n = e->list_plan_h[2 + 2 * t];
    int64_t N = e->list_plan_h[3 + 2 * t];
    if (N == 0) continue;
    if (e->list_out + N > e->cfg.out_capacity) return fail(e, FW_ERR_CAPACITY, "output log capacity exceeded (list state)");
    if (int rc = list_sort_window(e, n, N)) return rc;
    if (e->disarmed.count(n)) {   // a restored window that fired before the checkpoint: only the re-armed keys fire
      std::vector<int64_t> pos((size_t)N);
      std::vector<unsigned long long> kids((size_t)N);
      std::vector<uint8_t> armed((size_t)e->s.stride);
      const int32_t p = (int32_t)floor_mod(n, e->s.P);
      HIPCHK(e, hipMemcpyAsync(pos.data(), e->list_v1, 8 * (size_t)N, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(e, hipMemcpyAsync(kids.data(), e->list_k2, 8 * (size_t)N, hipMemcpyDeviceToHost, e->stream));
      HIPCHK(e, hipMemcpyAsync(armed.data(), e->s.armed + (size_t)p * (size_t)e->s.stride, (size_t)e->s.stride,
                               hipMemcpyDeviceToHost, e->stream));
      HIPCHK(e, hipStreamSynchronize(e->stream));
      int64_t keep = 0;
      for (int64_t x = 0; x < N; ++x)
        if (armed[(size_t)kids[(size_t)x]]) pos[(size_t)keep++] = pos[(size_t)x];
      N = keep;
      if (N == 0) continue;
      HIPCHK(e, hipMemcpyAsync(e->list_v1, pos.data(), 8 * (size_t)N, hipMemcpyHostToDevice, e->stream));
      HIPCHK(e, hipStreamSynchronize(e->stream));
    }
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((N + BLOCK - 1) / BLOCK, e->grid));
    const int64_t max_ts = jsub(jadd(jadd(e->s.offset, (int64_t)((uint64_t)n * (uint64_t)e->s.slide)), e->s.size), 1);
    hipLaunchKernelGGL(k_list_emit, dim3(blocks), dim3(BLOCK), 0, e->stream, e->s, e->lst, e->list_v1, N, e->list_out, max_ts);
    DBGSYNC(e, "k_list_emit");
    e->list_out += N;
  }
  hipLaunchKernelGGL(k_list_finish, dim3(1), dim3(1024), 0, e->stream, e->s, e->lst, e->list_plan, e->list_out);
  if (int rc = disarm_advance(e, wm)) return rc;
  DBGSYNC(e, "k_list_finish");
  hipLaunchKernelGGL(k_mark_only, dim3(1), dim3(1), 0, e->stream, e->s, wm);
  e->phase_end(e->s.stride);
  HIPCHK(e, hipGetLastError());
  e->hmarks.push_back({wm, e->dev_marks++, true});
  e->out_dirty = false;
  e->cur_wm = wm;
  return FW_OK;
}
