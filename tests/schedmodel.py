"""A serial per-packet model of the reference's delivery step and the slice of
its scheduler that delivery can reach, for checking the host post-pass
(gcl_host_deliver*) against rx.c packet by packet.

  rx_send_to_runtime      iokernel/rx.c:50-73
  rx_send_pkt_to_runtime  iokernel/rx.c:76-92
  rx_one_pkt's exits      iokernel/rx.c:171-232 (broadcast, ARP, fail_free)
  sched_steer_flows       iokernel/sched.c:122-147
  sched_enable_kthread    iokernel/sched.c:149-172 (appended to active_threads,
                          last_core = NCPU)
  sched_disable_kthread   iokernel/sched.c:174-192 (steers BEFORE the thread
                          leaves active_threads, as written; then the last
                          active thread is swapped into its index, :185-186)
  sched_pick_kthread      iokernel/sched.c:194-206 (a thread last parked on
                          this core or its hyperthread sibling first, else
                          list_tail of idle_threads)
  __sched_run             iokernel/sched.c:208-236: a core still waiting on its
                          last request disables the kthread pending on it --
                          a thread of ANY runtime -- so one runtime's wake can
                          re-steer another runtime, or take its last core,
                          in the middle of a burst
  sched_run_on_core       iokernel/sched.c:247-268

`Sched` is the scheduler state; the model reads it directly, and the C
post-pass sees it through the struct gcl_host_proc mirrors that `sync`
rewrites after every sched_add_core callback.  Test infrastructure only.
"""
import ctypes

import numpy as np

DELIVER, WAKE, DROP_ET, DROP_UNREG, BCAST, ARP_RESP = 0, 1, 2, 3, 4, 5


def steer(tc, active):
    """sched_steer_flows over the active_threads order (sched.c:122-147);
    None when no thread is active (the table is left as it was)."""
    if not active:
        return None
    flow = [0xFFFF] * tc
    for th in active:
        flow[th] = th
    j = 0
    for i in range(tc):
        if flow[i] == 0xFFFF:
            flow[i] = active[j % len(active)]
            j += 1
    return flow


NCPU = 256             # inc/base/limits.h: last_core of a running thread
UINT16_MAX = 0xFFFF    # last_core of a thread never parked (sched.c:898) or
                       # disabled by __sched_run's pending branch (:220)


def sibling(core):
    """sched_siblings[] of the model's host: hyperthread pairs (2k, 2k + 1)."""
    return core ^ 1


class Proc:
    def __init__(self, uniqid, tc, active, parked=None):
        self.uniqid, self.tc = uniqid, tc
        self.active = list(active)                        # p->active_threads order
        self.idle = [t for t in range(tc) if t not in self.active]  # head = list_top
        self.flow = steer(tc, self.active) or [0] * tc
        # p->last_core: NCPU while running; where an idle thread was parked
        # (@parked: thread -> core), else UINT16_MAX
        self.last_core = [NCPU if t in self.active else (parked or {}).get(t, UINT16_MAX)
                          for t in range(tc)]


class Sched:
    """Cores that are all still waiting on their last run request (s->wait),
    each with a pending kthread, so every sched_run_on_core goes down
    __sched_run's pending_th branch: the previous pending thread, of
    whatever runtime, is disabled."""

    def __init__(self, runtimes, ncores, rng):
        # idle kthreads parked earlier on cores of this host (sched_yield /
        # detach paths, sched_disable_kthread(th, core)), so that
        # sched_pick_kthread's last_core preference is exercised
        self.procs = {}
        for r in runtimes:
            idle = [t for t in range(r["thread_count"]) if t not in r["active_idx"]]
            parked = {t: int(rng.integers(0, ncores)) for t in idle if rng.random() < 0.5}
            self.procs[r["uniqid"]] = Proc(r["uniqid"], r["thread_count"], r["active_idx"], parked)
        running = [(u, th) for u, p in self.procs.items() for th in p.active]
        rng.shuffle(running)
        self.pending = [running[i] if i < len(running) else None for i in range(ncores)]
        self.rr = 0
        self.events = []

    def enable(self, p, th):
        p.last_core[th] = NCPU                     # sched.c:157
        p.idle.remove(th)
        p.active.append(th)                        # at_idx = active_thread_count++
        p.flow = steer(p.tc, p.active) or p.flow

    def disable(self, p, th, last_core=UINT16_MAX):
        p.last_core[th] = last_core                # sched.c:180
        p.idle.insert(0, th)                       # list_add: new head
        p.flow = steer(p.tc, p.active) or p.flow   # before the removal, sched.c:182-183
        i = p.active.index(th)                     # at_idx
        p.active[i] = p.active[-1]                 # sched.c:185-186: the last active
        p.active.pop()                             # thread moves into the hole

    @staticmethod
    def pick(p, core):
        """sched_pick_kthread (sched.c:194-206)."""
        for i in range(p.tc):
            if p.last_core[i] == core or p.last_core[i] == sibling(core):
                return i
        return p.idle[-1]                          # list_tail(&p->idle_threads)

    def add_core(self, u):
        """sched_add_core -> notify_core_needed -> sched_run_on_core(p, core)"""
        p = self.procs[u]
        self.events.append(("wake", u))
        if not p.idle:
            return  # sched_run_on_core: list_empty(&p->idle_threads) -> -EINVAL
        core = self.rr % len(self.pending)
        self.rr += 1
        th = self.pick(p, core)
        self.enable(p, th)
        prev = self.pending[core]
        if prev is not None and prev != (u, th):
            q = self.procs[prev[0]]
            if prev[1] in q.active:
                self.disable(q, prev[1], UINT16_MAX)  # __sched_run, sched.c:218-221
                self.events.append(("disable", prev[0], prev[1], len(q.active)))
        self.pending[core] = (u, th)

    def sync(self, cprocs):
        """Mirror the state into the struct gcl_host_proc the C post-pass reads."""
        for u, p in self.procs.items():
            c = cprocs[u]
            c.active_thread_count = len(p.active)
            c.idle_top = p.idle[0] if p.idle else -1
            for i, f in enumerate(p.flow):
                c.flow_tbl[i] = f


def rx_model(S, v8, client_order, ring_size, pkt_len, olflags, shmptr, bcast_hash, arp_ok):
    """rx.c's post-classification steps for each packet in order, against
    scheduler state S.  v8: the 8-B verdicts (action, uniqid and the hash
    rx_send_to_runtime takes: hash.rss, rx.c:83).  Returns (delivered,
    stats[8], events, rings{(u, th): [(cmd, payload)]})."""
    stats = [0] * 8
    rings = {(u, th): [] for u, p in S.procs.items() for th in range(p.tc)}
    events = S.events
    delivered = 0

    def send(u, h, cmd, payload):
        p = S.procs[u]
        if p.active:                                      # rx.c:55-59
            th = p.flow[h % p.tc]
        else:                                             # rx.c:62-72
            S.add_core(u)
            if not p.active:
                if not p.idle:
                    return False
                th = p.idle[0]
            else:
                th = p.flow[h % p.tc]
        events.append(("poll", u, th))
        if len(rings[(u, th)]) >= ring_size:
            return False
        rings[(u, th)].append((cmd, payload))
        return True

    for i in range(len(v8)):
        act = int(v8["action"][i]) & 0x3F
        cmd = int(pkt_len[i]) << 16 | ((int(olflags[i]) & 0x0C) == 0x08) << 48
        pay = int(shmptr[i])
        if act in (DELIVER, WAKE):
            u = int(v8["uniqid"][i])
            if send(u, int(v8["hash"][i]), cmd, pay):
                events.append(("own", u, i))
                delivered += 1
                continue
            stats[1] += 1                                 # RX_UNICAST_FAIL
        elif act == BCAST:                                # rx.c:171-190
            sent = 0
            for u in client_order:
                if send(u, int(bcast_hash[i]), cmd, pay):
                    sent += 1
                    events.append(("own", u, i))
                else:
                    stats[2] += 1                         # RX_BROADCAST_FAIL
            if sent == 0:
                events.append(("free", i))
            else:
                delivered += 1
                events.append(("ref", i, sent - 1))
            continue
        elif act == ARP_RESP:                             # rx.c:200-207
            events.append(("arp", i))
            if arp_ok(i):
                continue
            stats[0] += 1
        else:
            events.append(("free", i))                    # device-counted drops
            continue
        events.append(("free", i))                        # fail_free, rx.c:225-232
        stats[4] += 1
    return delivered, stats, events, rings


def make_cprocs(g, S, ring_size, ring_cls):
    """struct gcl_host_proc mirrors of S with one lrpc ring per kthread."""
    cprocs, rings = {}, {}
    for u, p in S.procs.items():
        c = g.GclHostProc()
        c.uniqid, c.thread_count = u, p.tc
        for th in range(p.tc):
            r = ring_cls(g, ring_size)
            rings[(u, th)] = r
            c.rxq[th] = ctypes.pointer(r.chan)
        cprocs[u] = c
    S.sync(cprocs)
    return cprocs, rings


def run_post_pass(g, S, cprocs, rings, form, verdicts, max_runtimes, client_order, pkt_len,
                  olflags, shmptr, bcast_hash, arp_ok, thread_bits=0):
    """Run one gcl_host_deliver* form over `verdicts` with callbacks driving S.
    form: 8, 4, 2, 1 (packed arrays) or "recs8"/.../"recs1" (loop records,
    `verdicts` then an array of LOOP_REC_DTYPE)."""
    events = S.events
    by_id = (ctypes.c_void_p * max_runtimes)()
    for u, c in cprocs.items():
        by_id[u] = ctypes.addressof(c)
    clients = (ctypes.c_void_p * len(client_order))(*[ctypes.addressof(cprocs[u])
                                                      for u in client_order])

    @g.SCHED_ADD_CORE_FN
    def add_core(arg, pp):
        S.add_core(pp.contents.uniqid)
        S.sync(cprocs)

    @g.FREE_PKT_FN
    def free_pkt(arg, i):
        events.append(("free", i))

    @g.REFCNT_FN
    def refcnt(arg, i, d):
        events.append(("ref", i, d))

    @g.OWNED_FN
    def owned(arg, pp, i):
        events.append(("own", pp.contents.uniqid, i))

    @g.ENABLE_POLL_FN
    def poll(arg, pp, th):
        events.append(("poll", pp.contents.uniqid, th))

    @g.ARP_RESPOND_FN
    def arp(arg, i):
        events.append(("arp", i))
        return arp_ok(i)

    ops = g.GclHostOps()
    ops.sched_add_core, ops.free_pkt, ops.refcnt_update = add_core, free_pkt, refcnt
    ops.owned, ops.enable_poll, ops.arp_respond = owned, poll, arp
    stats = np.zeros(8, dtype=np.uint64)
    n = len(verdicts)
    common = (pkt_len.ctypes.data, olflags.ctypes.data, 0x09, shmptr.ctypes.data, n,
              ctypes.byref(ops), stats.ctypes.data)
    bh = bcast_hash.ctypes.data
    if form == 8:
        d = g.lib.gcl_host_deliver(by_id, max_runtimes, clients, len(client_order),
                                   verdicts.ctypes.data, *common)
    elif form == 4:
        d = g.lib.gcl_host_deliver4(by_id, max_runtimes, clients, len(client_order),
                                    verdicts.ctypes.data, bh, *common)
    elif form == 2:
        d = g.lib.gcl_host_deliver2(by_id, max_runtimes, clients, len(client_order),
                                    verdicts.ctypes.data, thread_bits, bh, *common)
    elif form == 1:
        d = g.lib.gcl_host_deliver1(by_id, max_runtimes, clients, len(client_order),
                                    verdicts.ctypes.data, thread_bits, bh, *common)
    else:
        vb = int(form[4:])
        d = g.lib.gcl_host_deliver_recs(by_id, max_runtimes, clients, len(client_order),
                                        verdicts.ctypes.data, vb, thread_bits,
                                        bh if vb != 8 else None, *common)
    return d, [int(x) for x in stats], events, {k: r.drain() for k, r in rings.items()}


def loop_records(g, v8, v4, v2, vb, v1=None):
    """The rx loop's 16-B records (struct gcl_loop_rec) of these verdicts."""
    r = np.zeros(len(v8), dtype=g.LOOP_REC_DTYPE)
    r["ticket"] = 7
    if vb == 8:
        r["hash"], r["verdict"] = v8.view(np.uint64) & 0xFFFFFFFF, v8.view(np.uint64) >> 32
    else:
        r["hash"] = 0xDEADBEEF  # unused by the compact forms
        r["verdict"] = v4.view(np.uint32) if vb == 4 else v2.astype(np.uint32) if vb == 2 \
            else v1.astype(np.uint32)
    return r
