"""ctypes binding of the CPU oracle (oracle/liboracle.so).

*** TEST INFRASTRUCTURE ***  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module: it is the checker the
HIP path is compared against, never part of the product path.

Parity: pinned by the reference's own fixtures -- see
oracle/odp_cls_oracle.c's header and DESIGN.md ("Oracle").
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

RESULT_DTYPE = np.dtype([("in_flags", "<u4"), ("err", "u1"), ("outcome", "u1"), ("cos", "u1"),
                         ("hops", "u1"), ("queue", "<u2"), ("mark", "<u2"),
                         ("l3_offset", "<u2"), ("l4_offset", "<u2")])


class Term(C.Structure):
    _fields_ = [("term", C.c_int), ("value", C.c_uint8 * 16), ("mask", C.c_uint8 * 16),
                ("val_sz", C.c_uint32), ("offset", C.c_uint32)]


def build():
    """Compile the restatement if needed (gcc, seconds)."""
    src = os.path.join(HERE, "odp_cls_oracle.c")
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB)
        vp, i32, u32 = C.c_void_p, C.c_int, C.c_uint32
        L.orc_reset.argtypes = [u32, u32, u32]
        L.orc_cos_create.argtypes = [i32, u32, i32, u32, i32]
        L.orc_cos_create.restype = i32
        L.orc_cos_destroy.argtypes = [i32]
        L.orc_pmr_create.argtypes = [C.POINTER(Term), i32, u32, i32, i32]
        L.orc_pmr_create.restype = i32
        L.orc_pmr_destroy.argtypes = [i32]
        L.orc_default_cos_set.argtypes = [i32]
        L.orc_error_cos_set.argtypes = [i32]
        L.orc_cos_stats_packets.argtypes = [i32]
        L.orc_cos_stats_packets.restype = C.c_uint64
        L.orc_classify_batch.argtypes = [vp, vp, vp, u32, vp, u32]
        L.orc_classify_batch_mt.argtypes = [vp, vp, vp, u32, vp, u32, i32]
        L.orc_parse_one.argtypes = [vp, u32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint32),
                                    C.POINTER(C.c_uint16), C.POINTER(C.c_uint16),
                                    C.POINTER(C.c_uint16)]
        L.orc_rss_hash_one.argtypes = [vp, u32, u32]
        L.orc_rss_hash_one.restype = u32
        L.orc_softrss.argtypes = [C.POINTER(C.c_uint32), u32]
        L.orc_softrss.restype = u32
        L.orc_pktin_opt_set.argtypes = [C.c_uint64]
        L.orc_pktin_opt_set.restype = None
        L.orc_eval_counts.argtypes = [C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.orc_eval_counts.restype = None
        _lib = L
    return _lib


class Oracle:
    """Scalar model of linux-generic's classifier tables + data path."""

    def __init__(self, limits=(255, 8192, 4096), max_hops=None, pktin_opt=0):
        self.L = lib()
        self.L.orc_reset(*limits)
        self.max_hops = limits[0] if max_hops is None else max_hops
        self.cos = []
        self.pmr = []
        # odp_pktin_config_opt_t.all_bits (checksum validation / drop on error)
        self.pktin_opt = pktin_opt

    def cos_create(self, action=0, queue=1, num_queue=1, hash_proto=0, stats=0):
        return self.L.orc_cos_create(action, num_queue, 1 if queue else 0, hash_proto, stats)

    def pmr_create(self, terms, src, dst, mark=0):
        arr = (Term * max(1, len(terms)))()
        for i, (term, value, mask, offset) in enumerate(terms):
            arr[i].term = term
            for j, b in enumerate(bytes(value)[:16]):
                arr[i].value[j] = b
            for j, b in enumerate(bytes(mask)[:16]):
                arr[i].mask[j] = b
            arr[i].val_sz = len(value)
            arr[i].offset = offset
        return self.L.orc_pmr_create(arr, len(terms), mark, src, dst)

    def apply(self, prog):
        for op in prog:
            k = op[0]
            if k == "cos":
                a = op[2]
                self.cos.append(self.cos_create(a["action"], a["queue"], a["num_queue"],
                                                a["hash_proto"], a["stats"]))
            elif k == "pmr":
                self.pmr.append(self.pmr_create(op[1], self.cos[op[2]], self.cos[op[3]], op[4]))
            elif k == "pmr_destroy":
                self.L.orc_pmr_destroy(self.pmr[op[1]])
            elif k == "cos_destroy":
                self.L.orc_cos_destroy(self.cos[op[1]])
            elif k == "default":
                self.L.orc_default_cos_set(0 if op[1] is None else self.cos[op[1]])
            elif k == "error":
                self.L.orc_error_cos_set(0 if op[1] is None else self.cos[op[1]])
            else:
                raise ValueError(op)
        return self.cos, self.pmr

    def classify(self, batch, threads=1):
        n = batch.n
        out = np.zeros(max(1, n), dtype=RESULT_DTYPE)
        buf = np.ascontiguousarray(batch.buf)
        off = np.ascontiguousarray(batch.off, dtype=np.uint32)
        ln = np.ascontiguousarray(batch.len, dtype=np.uint16)
        self.L.orc_pktin_opt_set(self.pktin_opt)
        if threads == 1:
            self.L.orc_classify_batch(buf.ctypes.data, off.ctypes.data, ln.ctypes.data, n,
                                      out.ctypes.data, self.max_hops)
        else:
            self.L.orc_classify_batch_mt(buf.ctypes.data, off.ctypes.data, ln.ctypes.data, n,
                                         out.ctypes.data, self.max_hops, threads)
        return out[:n]

    def eval_counts(self, batch):
        """Classify ``batch`` on this thread and return the reference's
        linear-scan work for it: (PMRs verified, terms evaluated)."""
        r, t = C.c_uint64(), C.c_uint64()
        self.L.orc_eval_counts(C.byref(r), C.byref(t))   # reset
        self.classify(batch)
        self.L.orc_eval_counts(C.byref(r), C.byref(t))
        return r.value, t.value

    def stats_packets(self, cos_handle):
        return self.L.orc_cos_stats_packets(cos_handle)


def parse(frame: bytes, pktin_opt=0):
    """Parse one frame; returns (ret, input_flags, err, l2, l3, l4)."""
    L = lib()
    L.orc_pktin_opt_set(pktin_opt)
    b = np.frombuffer(frame + bytes(8), dtype=np.uint8)
    f, e = C.c_uint64(), C.c_uint32()
    l2, l3, l4 = C.c_uint16(), C.c_uint16(), C.c_uint16()
    r = L.orc_parse_one(b.ctypes.data, len(frame), C.byref(f), C.byref(e), C.byref(l2),
                        C.byref(l3), C.byref(l4))
    return r, f.value, e.value, l2.value, l3.value, l4.value
