"""ctypes binding of libodp_cls.so (include/odp_cls_api.h) and libmi_cls.so.

This is the host-side mirror of the reference's classifier interface
(include/odp/api/spec/classification.h) used by the tests and bench: the
same function names, argument meaning and error behaviour (INVALID handle
= 0 on failure, -1 from destroy, ...).  The compute path is the HIP kernel in
libmi_cls.so; there is no CPU fallback -- loading fails loudly if the
native libraries are missing.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import rules as R

_HERE = os.path.dirname(os.path.abspath(__file__))
# ODP_AMD_LIB_DIR selects an alternative build (kernel variants for A/B runs)
_LIBDIR = os.environ.get("ODP_AMD_LIB_DIR", _HERE)
LIB_MI = os.path.join(_LIBDIR, "libmi_cls.so")
LIB_ODP = os.path.join(_LIBDIR, "libodp_cls.so")


class PmrParam(C.Structure):
    """odp_pmr_param_t (classification.h:278-321)."""
    _fields_ = [("term", C.c_int), ("range_term", C.c_bool), ("value", C.c_void_p),
                ("mask", C.c_void_p), ("val_sz", C.c_uint32), ("offset", C.c_uint32)]


class PmrCreateOpt(C.Structure):
    """odp_pmr_create_opt_t."""
    _fields_ = [("terms", C.POINTER(PmrParam)), ("num_terms", C.c_int), ("mark", C.c_uint64),
                ("priority", C.c_uint32)]


class SchedParam(C.Structure):
    _fields_ = [("prio", C.c_int), ("sync", C.c_int), ("group", C.c_int),
                ("lock_count", C.c_uint32)]


class QueueParam(C.Structure):
    """odp_queue_param_t (queue_types.h:249-349)."""
    _fields_ = [("type", C.c_int), ("enq_mode", C.c_int), ("deq_mode", C.c_int),
                ("sched", SchedParam), ("order", C.c_int), ("nonblocking", C.c_int),
                ("context", C.c_void_p), ("context_len", C.c_uint32), ("size", C.c_uint32),
                ("num_aggr", C.c_uint32), ("aggr", C.c_void_p)]


class _QP(C.Structure):
    _fields_ = [("queue_param", QueueParam), ("hash_proto", C.c_uint32)]


class _QU(C.Union):
    _fields_ = [("queue", C.c_void_p), ("qp", _QP)]


class RedParam(C.Structure):
    _fields_ = [("enable", C.c_bool), ("threshold", C.c_uint64)]


class BpParam(C.Structure):
    _fields_ = [("enable", C.c_bool), ("threshold", C.c_uint64), ("pfc_level", C.c_uint8)]


class VectorCfg(C.Structure):
    _fields_ = [("enable", C.c_bool), ("pool", C.c_void_p), ("max_tmo_ns", C.c_uint64),
                ("max_size", C.c_uint32)]


class AggrProfile(C.Structure):
    _fields_ = [("type", C.c_int), ("param", C.c_void_p)]


class CosParam(C.Structure):
    """odp_cls_cos_param_t (classification.h:647-770)."""
    _anonymous_ = ("u",)
    _fields_ = [("action", C.c_int), ("stats_enable", C.c_bool), ("num_queue", C.c_uint32),
                ("u", _QU), ("pool", C.c_void_p), ("red", RedParam), ("bp", BpParam),
                ("vector", VectorCfg), ("aggr_enq_profile", AggrProfile)]


class CosStats(C.Structure):
    _fields_ = [("octets", C.c_uint64), ("packets", C.c_uint64), ("discards", C.c_uint64),
                ("errors", C.c_uint64)]


class Capability(C.Structure):
    _fields_ = [("supported_terms", C.c_uint64), ("max_pmr", C.c_uint32),
                ("max_pmr_per_cos", C.c_uint32), ("max_terms_per_pmr", C.c_uint32),
                ("max_pmr_priority", C.c_uint32), ("max_cos", C.c_uint32),
                ("max_cos_stats", C.c_uint32), ("max_hash_queues", C.c_uint32),
                ("hash_protocols", C.c_uint32), ("pmr_range_supported", C.c_bool),
                ("random_early_detection", C.c_int), ("threshold_red", C.c_uint8),
                ("back_pressure", C.c_int), ("threshold_bp", C.c_uint8),
                ("max_mark", C.c_uint64), ("stats_cos", C.c_uint64), ("stats_queue", C.c_uint64)]


def _load():
    for p in (LIB_MI, LIB_ODP):
        if not os.path.exists(p):
            raise RuntimeError(f"{p} is missing: run __graft_entry__.build() (no CPU fallback)")
    C.CDLL(LIB_MI, mode=C.RTLD_GLOBAL)
    lib = C.CDLL(LIB_ODP)
    vp, u32, i32 = C.c_void_p, C.c_uint32, C.c_int
    sig = {
        "odp_cls_cos_param_init": (None, [C.POINTER(CosParam)]),
        "odp_cls_capability": (i32, [C.POINTER(Capability)]),
        "odp_cls_cos_create": (vp, [C.c_char_p, C.POINTER(CosParam)]),
        "odp_cos_destroy": (i32, [vp]),
        "odp_cos_queue_set": (i32, [vp, vp]),
        "odp_cos_queue": (vp, [vp]),
        "odp_cls_cos_num_queue": (u32, [vp]),
        "odp_cls_cos_queues": (u32, [vp, C.POINTER(vp), u32]),
        "odp_cls_cos_stats": (i32, [vp, C.POINTER(CosStats)]),
        "odp_cls_pmr_param_init": (None, [C.POINTER(PmrParam)]),
        "odp_cls_pmr_create": (vp, [C.POINTER(PmrParam), i32, vp, vp]),
        "odp_cls_pmr_create_opt": (vp, [C.POINTER(PmrCreateOpt), vp, vp]),
        "odp_cls_pmr_destroy": (i32, [vp]),
        "odp_cls_cos_pool_set": (i32, [vp, vp]),
        "odp_cls_cos_pool": (vp, [vp]),
        "odp_cos_to_u64": (C.c_uint64, [vp]),
        "odp_pmr_to_u64": (C.c_uint64, [vp]),
        "odp_cls_print_all": (None, []),
        "odp_pktio_default_cos_set": (i32, [vp, vp]),
        "odp_pktio_error_cos_set": (i32, [vp, vp]),
        "odp_pktio_skip_set": (i32, [vp, u32]),
        "odp_pktio_headroom_set": (i32, [vp, u32]),
        "odp_amd_cls_limits_set": (i32, [u32, u32, u32]),
        "odp_amd_cls_reset": (None, []),
        "odp_amd_cls_pktio_create": (vp, [i32]),
        "odp_amd_cls_pktio_create_multi": (vp, [C.POINTER(i32), i32]),
        "odp_amd_cls_classify_host": (i32, [vp, vp, C.c_size_t, vp, vp, u32, vp, i32]),
        "mi_cls_shard": (i32, [vp, u32, u32, vp]),
        "mi_cls_host_alloc": (vp, [C.c_size_t]),
        "mi_cls_host_free": (None, [vp]),
        "odp_amd_cls_pktio_destroy": (i32, [vp]),
        "odp_amd_cls_compile": (C.c_long, [vp, vp, C.c_size_t]),
        "odp_amd_cls_classify": (i32, [vp, vp, vp, vp, u32, vp, vp]),
        "odp_amd_cls_queue_of": (vp, [u32, u32]),
        "odp_amd_cls_generation": (C.c_uint64, []),
        "odp_amd_cls_pktin_opt_set": (i32, [vp, C.c_uint64]),
        "odp_amd_cls_spec_wait": (i32, [vp]),
        "mi_cls_spec_wait": (i32, [vp]),
        "odp_amd_cls_last_launch": (i32, [vp, C.POINTER(u32), u32]),
        "mi_cls_last_launch": (i32, [vp, C.POINTER(u32), u32]),
        "mi_cls_spec_pending": (i32, [C.POINTER(u32), C.POINTER(u32), C.POINTER(u32)]),
        "mi_cls_device_count": (i32, []),
        "mi_cls_ctx_create": (i32, [i32, C.POINTER(vp)]),
        "mi_cls_ctx_destroy": (i32, [vp]),
        "mi_cls_rules_load": (i32, [vp, vp, C.c_size_t, vp]),
        "mi_cls_classify": (i32, [vp, vp, vp, vp, u32, vp, vp]),
        "mi_cls_strerror": (C.c_char_p, [i32]),
        "mi_cls_program_info": (i32, [vp, C.c_size_t, C.POINTER(u32), u32]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


_lib = None


def shard(lens: np.ndarray, nshards: int) -> np.ndarray:
    """mi_cls_shard: begin[0..nshards] of contiguous slices balanced by
    header-window bytes (the product's multi-GPU cut; host only)."""
    ln = np.ascontiguousarray(lens, dtype=np.uint16)
    begin = np.zeros(nshards + 1, dtype=np.uint32)
    rc = lib().mi_cls_shard(ln.ctypes.data, int(ln.shape[0]), nshards, begin.ctypes.data)
    if rc:
        raise RuntimeError(f"mi_cls_shard: {rc}")
    return begin


class PinnedArray:
    """numpy view of page-locked host memory from mi_cls_host_alloc
    (hipHostMalloc): the GPU reads and writes it in place (zero copy)."""

    def __init__(self, nbytes: int):
        self.ptr = lib().mi_cls_host_alloc(max(1, nbytes))
        if not self.ptr:
            raise MemoryError("mi_cls_host_alloc failed")
        self.nbytes = nbytes
        self.u8 = np.ctypeslib.as_array((C.c_uint8 * max(1, nbytes)).from_address(self.ptr))

    def view(self, dtype, count=None):
        a = self.u8.view(dtype)
        return a if count is None else a[:count]

    def close(self):
        if self.ptr:
            lib().mi_cls_host_free(self.ptr)
            self.ptr = None


def spec_pending() -> dict:
    """Specialised-kernel compiler state (mi_cls_spec_pending)."""
    r, q, c = C.c_uint32(), C.c_uint32(), C.c_uint32()
    active = lib().mi_cls_spec_pending(C.byref(r), C.byref(q), C.byref(c))
    return {"active": bool(active), "running": r.value, "queued": q.value, "cached": c.value}


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def _h(x):
    return x or 0


class Classifier:
    """One classifier-enabled receive endpoint (pktio) on one GPU, driven
    through the ODP classification API.  ``apply(program)`` replays a rule
    program (odp_amd.rules) with odp_cls_* calls."""

    def __init__(self, gpu: int = 0, limits=(255, 8192, 4096), gpus=None):
        """gpus: a list of device ids -- host batches (classify_host) are then
        sharded over them (mi_cls_group_classify_host)."""
        L = lib()
        L.odp_amd_cls_reset()
        if limits is not None:
            assert L.odp_amd_cls_limits_set(*limits) == 0
        self.L = L
        if gpus:
            arr = (C.c_int * len(gpus))(*gpus)
            self.pktio = L.odp_amd_cls_pktio_create_multi(arr, len(gpus))
        else:
            self.pktio = L.odp_amd_cls_pktio_create(gpu)
        if not self.pktio:
            raise RuntimeError("odp_amd_cls_pktio_create failed")
        self.cos = []
        self.pmr = []
        self._keep = []

    def close(self):
        if self.pktio:
            self.L.odp_amd_cls_pktio_destroy(self.pktio)
            self.pktio = None

    # -- API passthroughs ------------------------------------------------
    def cos_create(self, name, action=0, queue=1, num_queue=1, hash_proto=0, stats=0, pool=0):
        p = CosParam()
        self.L.odp_cls_cos_param_init(C.byref(p))
        p.action = action
        p.num_queue = num_queue
        p.stats_enable = bool(stats)
        if num_queue > 1:
            p.qp.hash_proto = hash_proto
        else:
            p.queue = queue
        p.pool = pool
        return _h(self.L.odp_cls_cos_create(name.encode() if name else None, C.byref(p)))

    def _terms(self, terms):
        arr = (PmrParam * max(1, len(terms)))()
        keep = []
        for i, (term, value, mask, offset) in enumerate(terms):
            vb = C.create_string_buffer(bytes(value), max(1, len(value)))
            mb = C.create_string_buffer(bytes(mask), max(1, len(mask)))
            keep += [vb, mb]
            arr[i].term = term
            arr[i].range_term = False
            arr[i].value = C.cast(vb, C.c_void_p)
            arr[i].mask = C.cast(mb, C.c_void_p)
            arr[i].val_sz = len(value)
            arr[i].offset = offset
        return arr, keep

    def pmr_create(self, terms, src, dst, mark=0):
        arr, keep = self._terms(terms)
        if mark:
            o = PmrCreateOpt()
            o.terms = C.cast(arr, C.POINTER(PmrParam))
            o.num_terms = len(terms)
            o.mark = mark
            o.priority = 0
            return _h(self.L.odp_cls_pmr_create_opt(C.byref(o), src, dst))
        return _h(self.L.odp_cls_pmr_create(C.cast(arr, C.POINTER(PmrParam)), len(terms), src, dst))

    def apply(self, prog):
        """Replay a rule program; returns (cos handles, pmr handles)."""
        for op in prog:
            k = op[0]
            if k == "cos":
                a = op[2]
                self.cos.append(self.cos_create(op[1], action=a["action"], queue=a["queue"],
                                                num_queue=a["num_queue"],
                                                hash_proto=a["hash_proto"], stats=a["stats"]))
            elif k == "pmr":
                self.pmr.append(self.pmr_create(op[1], self.cos[op[2]], self.cos[op[3]], op[4]))
            elif k == "pmr_destroy":
                self.L.odp_cls_pmr_destroy(self.pmr[op[1]])
            elif k == "cos_destroy":
                self.L.odp_cos_destroy(self.cos[op[1]])
            elif k == "default":
                self.L.odp_pktio_default_cos_set(self.pktio, 0 if op[1] is None else self.cos[op[1]])
            elif k == "error":
                self.L.odp_pktio_error_cos_set(self.pktio, 0 if op[1] is None else self.cos[op[1]])
            else:
                raise ValueError(op)
        return self.cos, self.pmr

    def set_pktin_opt(self, opt: int):
        """pktin parse options of this receive endpoint
        (odp_pktin_config_opt_t.all_bits: bits 2-5 IPv4/UDP/TCP/SCTP
        checksum validation, bits 6-10 drop on IPv4/IPv6/UDP/TCP/SCTP
        errors)."""
        assert self.L.odp_amd_cls_pktin_opt_set(self.pktio, int(opt)) == 0

    def compile(self) -> bytes:
        n = self.L.odp_amd_cls_compile(self.pktio, None, 0)
        buf = C.create_string_buffer(n)
        assert self.L.odp_amd_cls_compile(self.pktio, buf, n) == n
        return buf.raw

    def program_info(self) -> dict:
        """Device encoding of the current rule snapshot (host only)."""
        blob = self.compile()
        info = (C.c_uint32 * 13)()
        rc = self.L.mi_cls_program_info(blob, len(blob), info, 13)
        if rc:
            raise RuntimeError(f"mi_cls_program_info: {rc}")
        return {"words": info[0], "hot_words": info[1], "blocks": info[2],
                "direct": info[3], "candidate": info[4], "bitmap": info[5], "wide": info[6],
                "tree": bool(info[7]), "cand1": info[8], "flat_engine": int(info[9]) - 1,
                "chained": info[10], "joint_direct": info[11], "joint_bitmap": info[12]}

    def spec_wait(self) -> int:
        """Snapshot the rules and wait for their program-specialised kernel
        (odp_amd_cls_spec_wait): 0 in use, 1 none (not a flat program,
        MI_CLS_JIT=0, or the compile failed)."""
        rc = self.L.odp_amd_cls_spec_wait(self.pktio)
        if rc < 0:
            raise RuntimeError(f"odp_amd_cls_spec_wait: {rc}")
        return rc

    def last_launch(self) -> dict:
        """The kernel instantiation of the last device launch
        (odp_amd_cls_last_launch)."""
        info = (C.c_uint32 * 7)()
        rc = self.L.odp_amd_cls_last_launch(self.pktio, info, 7)
        if rc < 0:
            raise RuntimeError(f"odp_amd_cls_last_launch: {rc}")
        k = {"nw": info[0], "lds_hot": bool(info[1]), "div": bool(info[2]),
             "flat_engine": int(info[3]) - 1, "specialised": bool(info[4]), "ck": bool(info[5]),
             "grid": info[6]}
        k["name"] = (f"mi_cls_kernel<LT={int(k['lds_hot'])}, DIV={int(k['div'])}, NW={k['nw']}, "
                     f"FM={k['flat_engine']}, CK={int(k['ck'])}"
                     f"{', MiSpec' if k['specialised'] else ''}>")
        return k

    # -- data path -------------------------------------------------------
    def classify_device(self, d_buf, d_off, d_len, n, d_out, stream=0):
        """Batch classify on device pointers (ints).  Returns the C status."""
        return self.L.odp_amd_cls_classify(self.pktio, d_buf, d_off, d_len, n, d_out, stream)

    def classify(self, batch, device="cuda:0"):
        """Convenience: upload a pktgen.Batch, classify, return a numpy
        structured array of result records (RESULT_DTYPE)."""
        import torch
        dev = torch.device(device)
        t_buf = torch.from_numpy(np.ascontiguousarray(batch.buf)).to(dev)
        t_off = torch.from_numpy(batch.off.astype(np.int32, copy=False).view(np.int32)).to(dev)
        t_len = torch.from_numpy(batch.len.astype(np.int16, copy=False).view(np.int16)).to(dev)
        t_out = torch.empty((max(1, batch.n), 4), dtype=torch.int32, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        rc = self.classify_device(t_buf.data_ptr(), t_off.data_ptr(), t_len.data_ptr(), batch.n,
                                  t_out.data_ptr(), stream)
        if rc != 0:
            raise RuntimeError(f"odp_amd_cls_classify: {rc} "
                               f"({self.L.mi_cls_strerror(rc).decode()})")
        torch.cuda.synchronize(dev)
        out = t_out.cpu().numpy().view(np.uint8).reshape(-1)[: 16 * batch.n]
        return out.view(R.RESULT_DTYPE).copy()

    def classify_host(self, batch):
        """The pktio receive-path entry (odp_amd_cls_classify_host): the
        batch from host memory, staged, classified (sharded over the
        pktio's GPUs when it has several) and the records copied back."""
        out = np.zeros(max(1, batch.n), dtype=R.RESULT_DTYPE)
        buf = np.ascontiguousarray(batch.buf)
        off = np.ascontiguousarray(batch.off, dtype=np.uint32)
        ln = np.ascontiguousarray(batch.len, dtype=np.uint16)
        rc = self.L.odp_amd_cls_classify_host(self.pktio, buf.ctypes.data, buf.nbytes,
                                              off.ctypes.data, ln.ctypes.data, batch.n,
                                              out.ctypes.data, 0)
        if rc != 0:
            raise RuntimeError(f"odp_amd_cls_classify_host: {rc}")
        return out[: batch.n]

    def cos_stats_packets(self, cos_handle):
        s = CosStats()
        assert self.L.odp_cls_cos_stats(cos_handle, C.byref(s)) == 0
        return s.packets
