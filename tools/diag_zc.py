"""Zero-copy check: classify one batch with inputs / records in device memory
and in page-locked host memory (every combination) and compare the records
with the oracle's.  Diagnostic tool, run on the GPU box."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from odp_amd import cls, rules as R   # noqa: E402
from oracle.oracle import Oracle      # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
mk = {2: R.config2, 3: R.config3, 4: R.config4, 5: R.config5}
b, p = mk[cfg](n)
o = Oracle()
o.apply(p)
exp = o.classify(b, threads=16)
c = cls.Classifier(gpu=0)
c.apply(p)
dev = torch.device("cuda:0")
sp = torch.cuda.current_stream(dev).cuda_stream
d_buf = torch.from_numpy(np.ascontiguousarray(b.buf)).to(dev)
d_off = torch.from_numpy(b.off.view(np.int32)).to(dev)
d_len = torch.from_numpy(b.len.view(np.int16)).to(dev)
d_out = torch.empty((b.n, 4), dtype=torch.int32, device=dev)
hb = cls.PinnedArray(b.buf.nbytes + 64)
ho = cls.PinnedArray(4 * b.n)
hl = cls.PinnedArray(2 * b.n)
hr = cls.PinnedArray(16 * b.n)
hb.u8[: b.buf.nbytes] = b.buf
ho.view(np.uint32)[:] = b.off
hl.view(np.uint16)[:] = b.len

for name, ins, out_host in (("dev/dev", (d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr()), False),
                            ("dev/host", (d_buf.data_ptr(), d_off.data_ptr(), d_len.data_ptr()), True),
                            ("host/dev", (hb.ptr, ho.ptr, hl.ptr), False),
                            ("host/host", (hb.ptr, ho.ptr, hl.ptr), True)):
    for rep in range(3):
        hr.u8[:] = 0xEE
        d_out.fill_(-1)
        assert c.classify_device(*ins, b.n, hr.ptr if out_host else d_out.data_ptr(), sp) == 0
        torch.cuda.synchronize(dev)
        if out_host:
            got = hr.u8[: 16 * b.n].copy().view(R.RESULT_DTYPE)
        else:
            got = d_out.cpu().numpy().view(np.uint8).reshape(-1).view(R.RESULT_DTYPE)
        bad = np.nonzero(got != exp)[0]
        print(name, rep, "mismatches", len(bad), flush=True)
        for i in bad[:4]:
            print("   pkt", i, "len", int(b.len[i]), "got", got[i], "exp", exp[i])
for a in (hb, ho, hl, hr):
    a.close()
c.close()
