"""Helpers for the runtime / receive-path tests: pcap writers, the rule
program text format read by tests/rt/rx_driver.c, the driver runner, and
the expected per-queue packet sequences derived from the CPU oracle with the
reference's receive-path rules (platform/linux-generic/pktio/loop.c:253-384,
pcap.c:280-401, include/odp_classification_internal.h:142-236)."""
from __future__ import annotations

import os
import struct
import subprocess
from collections import defaultdict

from odp_amd import pktgen as pg
from odp_amd import rules as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "tests", "_bin", "rx_driver")
EXAMPLE = os.path.join(ROOT, "examples", "_bin", "odp_classifier")

# input_flags bits the driver reconstructs from the odp_packet_has_*() calls
# (bit 0 cls_mark is reported through odp_packet_cls_mark, bits 20/21/26 have
# no accessor)
FLAG_MASK = sum(1 << b for b in list(range(1, 20)) + [22, 23, 24, 25])


# ------------------------------------------------------------------ pcap files
def write_pcap(path, frames, byteorder="<", nsec=False):
    """Classic libpcap file, DLT_EN10MB."""
    magic = 0xa1b23c4d if nsec else 0xa1b2c3d4
    with open(path, "wb") as f:
        f.write(struct.pack(byteorder + "IHHiIII", magic, 2, 4, 0, 0, 65535, 1))
        for i, fr in enumerate(frames):
            f.write(struct.pack(byteorder + "IIII", 1700000000 + i, i, len(fr), len(fr)))
            f.write(fr)


def write_pcapng(path, frames, byteorder="<"):
    """pcapng: SHB + IDB + one EPB per frame."""
    def block(btype, body):
        body += bytes((-len(body)) % 4)
        n = 12 + len(body)
        return struct.pack(byteorder + "II", btype, n) + body + struct.pack(byteorder + "I", n)
    with open(path, "wb") as f:
        f.write(block(0x0a0d0d0a, struct.pack(byteorder + "IHHq", 0x1a2b3c4d, 1, 0, -1)))
        f.write(block(1, struct.pack(byteorder + "HHI", 1, 0, 65535)))
        for i, fr in enumerate(frames):
            f.write(block(6, struct.pack(byteorder + "IIIII", 0, 0, i, len(fr), len(fr)) + fr))


# ------------------------------------------------------------------ rule text
def write_rules(path, prog):
    lines = []
    for op in prog:
        k = op[0]
        if k == "cos":
            a = op[2]
            assert " " not in op[1]
            lines.append(f"cos {op[1]} {a['action']} {a['num_queue']} {a['hash_proto']} "
                         f"{a['stats']}")
        elif k == "pmr":
            terms = op[1]
            parts = [f"pmr {op[2]} {op[3]} {op[4]} {len(terms)}"]
            for term, val, mask, off in terms:
                parts.append(f"{term} {val.hex() or '-'} {mask.hex() or '-'} {off}")
            lines.append(" ".join(parts))
        elif k in ("pmr_destroy", "cos_destroy"):
            lines.append(f"{k} {op[1]}")
        elif k in ("default", "error"):
            lines.append(f"{k} {-1 if op[1] is None else op[1]}")
        else:
            raise ValueError(op)
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


# ------------------------------------------------------------------ driver
def run_driver(pktio, rules_path, mode="sched", layer=4, cos_pools=1, cls=1, src=None,
               env=None, timeout=120, events=None):
    """events: a dict that receives, per queue, the delivery structure in
    order -- ("P",) a plain packet, ("V", n) / ("E", n) a packet / event
    vector of n packets (its packets are in the queue's packet list)."""
    args = [DRIVER, pktio, rules_path or "-", mode, str(layer), str(cos_pools), str(cls)]
    if src:
        args.append(src)
    e = dict(os.environ)
    e.update(env or {})
    try:
        r = subprocess.run(args, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                           timeout=timeout, env=e)
    except subprocess.TimeoutExpired as t:
        # the driver's phase markers (stderr "T ...") and its last output say
        # where it stopped
        err = (t.stderr or b"")[-2000:]
        out = (t.stdout or b"")[-600:]
        raise AssertionError(f"rx_driver timed out after {timeout} s: {' '.join(args)}\n"
                             f"stderr tail: {err!r}\nstdout tail: {out!r}") from None
    assert r.returncode == 0, f"rx_driver rc={r.returncode}\n{r.stderr[-2000:]}"
    queues = defaultdict(list)
    stats = None
    qstats = {}
    inside = defaultdict(int)   # packets still expected inside the last vector
    for line in r.stdout.splitlines():
        p = line.split()
        if not p:
            continue
        assert p[0] != "SEGMENTED", line
        if p[0] in ("V", "E"):
            if events is not None:
                events.setdefault(p[1], []).append((p[0], int(p[2])))
            inside[p[1]] = int(p[2])
            continue
        if p[0] == "P":
            if inside[p[1]]:
                inside[p[1]] -= 1
            elif events is not None:
                events.setdefault(p[1], []).append(("P",))
            q, pool, fl, err, l3, l4, mark, ln, data = p[1:10]
            queues[q].append((pool, int(fl, 16), int(err), int(l3), int(l4), int(mark),
                              int(ln), data))
        elif p[0] == "S":
            stats = tuple(int(x) for x in p[1:5])
        elif p[0] == "Q":
            qstats[(p[1], int(p[2]))] = (int(p[3]), int(p[4]))
    return dict(queues), stats, qstats


# ------------------------------------------------------------------ expectation
def cos_names(prog):
    """CoS slot -> (name, attrs) after replaying the program's creates and
    destroys with the lowest-free-slot rule (odp_classification.c:292-295)."""
    slots, refs = {}, []
    for op in prog:
        if op[0] == "cos":
            s = 0
            while s in slots:
                s += 1
            slots[s] = (op[1], op[2])
            refs.append(s)
        elif op[0] == "cos_destroy":
            slots.pop(refs[op[1]], None)
    return slots


def expected(prog, frames, cos_pools=1, cls=1, layer=4, pktin_queue="odp-pktin-0-0",
             pktin_opt=0):
    """Per-queue packet sequences and pktio stats the reference receive path
    produces, from the oracle's per-frame records.  pktin_opt: the pktio's
    odp_pktin_config_opt_t bits (the L3 layer takes only the IPv4 checksum
    and the IP drops, L2 none: odp_parse.c:372-414 stop before the rest)."""
    from oracle.oracle import Oracle
    if cls:
        layer = 4   # the classifier parses every layer (odp_packet_io.c:675-677)
    if layer == 2:
        pktin_opt &= (1 << 2) | (1 << 6) | (1 << 7)
    elif layer < 2:
        pktin_opt = 0
    o = Oracle(pktin_opt=pktin_opt)
    o.apply(prog if cls else [])
    recs = o.classify(pg.batch_from_frames(frames))
    slots = cos_names(prog) if cls else {}
    queues = defaultdict(list)
    qstats = defaultdict(lambda: [0, 0])
    in_pk = in_err = in_disc = octets = 0
    l2m = (1 << 3) | (0x3f << 6)
    l3m = l2m | (1 << 4) | (0x7f << 12) | (1 << 30)
    for fr, r in zip(frames, recs):
        fl, err, out = int(r["in_flags"]), int(r["err"]), int(r["outcome"])
        l3, l4 = int(r["l3_offset"]), int(r["l4_offset"])
        if layer == 0:
            fl, err, l3, l4 = 0, 0, 0xFFFF, 0xFFFF
        elif layer < 3:     # L2 (1) and L3 (2) cut the parse (odp_parse.c:372-414)
            if out == R.OUT_PARSE_DROP and not (layer == 2 and err & 2):
                out = R.OUT_DISCARD
            if layer == 1:
                fl, err, l4 = fl & l2m, err & 1, 0xFFFF
            else:
                fl, err = fl & l3m, err & 7
        if layer and (err or out == R.OUT_PARSE_DROP):
            in_err += 1
        if layer and out == R.OUT_PARSE_DROP:
            continue
        pool = "pktio_pool"
        if cls:
            if out in (R.OUT_DISCARD, R.OUT_LOOP):
                in_disc += 1
            if out != R.OUT_ENQ:
                continue
            name, attrs = slots[int(r["cos"])]
            if cos_pools:
                pool = name[:24] + "Pool"
            q = name if attrs["num_queue"] == 1 else f"_odp_cos_hq_{int(r['cos'])}_{int(r['queue'])}"
            qstats[(name, int(r["queue"]))][0] += 1
        else:
            q = pktin_queue
        if not err:
            in_pk += 1
            octets += len(fr)
        mark = int(r["mark"]) if (fl & 1) else 0
        # checksum statuses as the driver reports them (0 unknown, 1 bad, 2 ok)
        l3st = 0 if not (fl >> 30) & 1 else (1 if err & 4 else 2)
        l4st = 0 if not (fl >> 31) & 1 else (1 if err & 64 else 2)
        fl_rep = (fl & FLAG_MASK) | (l3st << 40) | (l4st << 42)
        queues[q].append((pool, fl_rep, int(err != 0), l3, l4, mark, len(fr), fr.hex()))
    return dict(queues), (in_pk, in_err, in_disc, octets), dict(qstats)


def expected_vectors(prog, frames, burst, max_size):
    """Per queue, the packet-vector delivery the receive path makes with
    packet vectors on every enqueue CoS (_odp_cos_enq / _odp_cos_vector_enq,
    odp_classification_internal.h:83-167): frames arrive in bursts of `burst`;
    inside a burst, consecutive enqueued packets with the same queue and CoS
    form a run (dropped packets do not end one; a burst's end does); a run of
    one is a plain packet, a longer run ceil(L / max_size) vectors, all full
    but the last."""
    from oracle.oracle import Oracle
    o = Oracle()
    o.apply(prog)
    recs = o.classify(pg.batch_from_frames(frames))
    slots = cos_names(prog)
    ev = defaultdict(list)

    def flush(key, n):
        if not n:
            return
        q = key[0]
        if n == 1:
            ev[q].append(("P",))
            return
        while n:
            k = min(n, max_size)
            ev[q].append(("V", k))
            n -= k

    for b0 in range(0, len(frames), burst):
        key, n = None, 0
        for r in recs[b0: b0 + burst]:
            if int(r["outcome"]) != R.OUT_ENQ:
                continue
            name, attrs = slots[int(r["cos"])]
            q = name if attrs["num_queue"] == 1 else f"_odp_cos_hq_{int(r['cos'])}_{int(r['queue'])}"
            k = (q, int(r["cos"]))
            if k != key:
                flush(key, n) if key else None
                key, n = k, 0
            n += 1
        if key:
            flush(key, n)
    return dict(ev)


def compare(got, exp):
    gq, gs, gqs = got
    eq, es, eqs = exp
    assert sorted(gq) == sorted(eq), (sorted(gq), sorted(eq))
    for q in eq:
        g, e = gq[q], eq[q]
        assert len(g) == len(e), (q, len(g), len(e))
        for i, (a, b) in enumerate(zip(g, e)):
            assert a == b, f"queue {q} packet {i}:\n  got {a[:7]}\n  exp {b[:7]}\n  frame {b[7]}"
    assert gs == es, (gs, es)
    for k, v in eqs.items():
        assert gqs.get(k, (0, 0))[0] == v[0], (k, gqs.get(k), v)


def pcap_frames(frames):
    """Frames the pcap path can carry: non-empty, within the pool's 1856 B."""
    return [f for f in frames if 0 < len(f) <= 1856]
