"""A small pure-Python restatement of event-time session windows (test infrastructure): the merging branch
of WindowOperator.processElement (WindowOperator.java:228-301), MergingWindowSet.addWindow
(MergingWindowSet.java:142-214), TimeWindow.mergeWindows (TimeWindow.java:186-230), EventTimeTrigger
(onElement :37-45, onEventTime :48-52, onMerge :70-74), PurgingTrigger (:44-76), cleanup (:420-428) and the
heap timer service's set semantics (a timer is (key, window, time); registering twice keeps one).

It is a second, independent statement of the semantics the C++ oracle restates, used on random streams
where the reference's own tests (tests/golden/session_*.json) give no known answers.  Integer sum and
count only (the fields whose result does not depend on the state window a merge picks).
"""
LONG_MAX = (1 << 63) - 1


class SessionModel:
    def __init__(self, gap, lateness=0, purging=False):
        self.gap, self.lateness, self.purging = gap, lateness, purging
        self.wm = -(1 << 63)
        self.windows = {}   # key -> {(start, end): [sum, count]}
        self.timers = set()  # (key, (start, end), time)
        self.out = []        # (key, sum, count, max_ts, start)
        self.marks = []      # (wm, position)

    def cleanup_time(self, w):
        ct = w[1] - 1 + self.lateness
        return ct if ct >= w[1] - 1 else LONG_MAX

    def element(self, key, ts, value):
        ws = self.windows.setdefault(key, {})
        w = (ts, ts + self.gap)
        # the new window's group: every in-flight window connected to it through intersections
        group, cover = [], w
        grew = True
        while grew:
            grew = False
            for x in list(ws):
                if x not in group and cover[0] <= x[1] and cover[1] >= x[0]:
                    group.append(x)
                    cover = (min(cover[0], x[0]), max(cover[1], x[1]))
                    grew = True
        if not group:
            actual, acc = w, None
        elif len(group) == 1 and group[0] == cover:
            actual, acc = cover, ws[cover]
        else:
            actual = cover
            acc = [0, 0]
            for x in group:   # merge: states folded, the merged windows' timers deleted
                s, c = ws.pop(x)
                acc[0] = (acc[0] + s + (1 << 63)) % (1 << 64) - (1 << 63)
                acc[1] += c
                self.timers.discard((key, x, x[1] - 1))
                self.timers.discard((key, x, self.cleanup_time(x)))
            ws[actual] = acc
            self.timers.add((key, actual, actual[1] - 1))   # onMerge
        if self.cleanup_time(actual) <= self.wm:   # isLate -> retireWindow
            ws.pop(actual, None)
            return
        if acc is None:
            acc = ws[actual] = [0, 0]
        acc[0] = (acc[0] + value + (1 << 63)) % (1 << 64) - (1 << 63)
        acc[1] += 1
        if actual[1] - 1 <= self.wm:   # onElement: FIRE
            self.out.append((key, acc[0], acc[1], actual[1] - 1, actual[0]))
            if self.purging:
                ws.pop(actual)
                self.timers.discard((key, actual, actual[1] - 1))
                return
        else:
            self.timers.add((key, actual, actual[1] - 1))
        self.timers.add((key, actual, self.cleanup_time(actual)))   # registerCleanupTimer

    def watermark(self, wm):
        self.wm = wm
        due = sorted((t for t in self.timers if t[2] <= wm), key=lambda t: t[2])
        for t in due:
            if t not in self.timers:
                continue
            self.timers.discard(t)
            key, w, time = t
            ws = self.windows.get(key, {})
            if w not in ws:
                continue   # purged: a leftover cleanup timer
            acc = ws[w]
            fire = time == w[1] - 1
            if fire:
                self.out.append((key, acc[0], acc[1], w[1] - 1, w[0]))
            if (fire and self.purging) or time == self.cleanup_time(w):
                ws.pop(w)
                self.timers.discard((key, w, w[1] - 1))
        self.marks.append((wm, len(self.out)))

    def epochs(self):
        ep, pos = [], 0
        for wm, mp in self.marks:
            ep.append((wm, sorted(self.out[pos:mp])))
            pos = mp
        if pos < len(self.out):
            ep.append(("tail", sorted(self.out[pos:])))
        return ep
