"""ODP runtime subset on the CPU (no GPU needed): pcap / pcapng reader, the
pcap promisc filter and loops= semantics, loop pktio, DIRECT / SCHED / QUEUE
input modes with the parser off (layer NONE needs no device), runtime unit
checks (tests/rt/rt_unit.c), and that the reference's example/classifier
binary links against this build and fails loudly without a GPU.

Reference behaviour: platform/linux-generic/pktio/pcap.c:90-401,
pktio/loop.c:253-384, odp_packet_io.c:650-715.
"""
import os
import subprocess

import pytest

from tests import rt_helpers as H
from tests import zoo

GOLD = os.path.join(H.ROOT, "tests", "golden")
UDP64 = os.path.join(GOLD, "udp64.pcap")


def _frames(q):
    return [bytes.fromhex(p[7]) for p in q]


def test_pcapng_reader_udp64(built):
    """example/classifier/udp64.pcap (pcapng) -> the 200 frames of the
    committed golden vector, in file order."""
    got, st, _ = H.run_driver(f"pcap:in={UDP64}", None, "direct", layer=0, cls=0)
    assert _frames(got["pktin"]) == zoo.udp64_frames()
    assert st == (200, 0, 0, 200 * 60)


@pytest.mark.parametrize("fmt", ["pcap_le", "pcap_be", "pcap_ns", "pcapng_le", "pcapng_be"])
def test_pcap_formats(built, tmp_path, fmt):
    frames = H.pcap_frames([f for _, f in zoo.all_frames()])
    p = str(tmp_path / "in.pcap")
    if fmt.startswith("pcapng"):
        H.write_pcapng(p, frames, "<" if fmt.endswith("le") else ">")
    else:
        H.write_pcap(p, frames, ">" if fmt == "pcap_be" else "<", nsec=fmt == "pcap_ns")
    got, st, _ = H.run_driver(f"pcap:in={p}", None, "direct", layer=0, cls=0)
    assert _frames(got["pktin"]) == frames


@pytest.mark.parametrize("loops,reads", [(1, 1), (2, 1), (3, 2), (5, 4)])
def test_pcap_loops(built, loops, reads):
    """_pcapif_reopen (pcap.c:257-278): loop_cnt starts at 1 and the file is
    re-read while ++loop_cnt < loops, so loops=N reads it max(1, N-1) times."""
    got, st, _ = H.run_driver(f"pcap:in={UDP64}:loops={loops}", None, "sched", layer=0, cls=0)
    assert len(got["odp-pktin-0-0"]) == 200 * reads


def test_pcap_promisc_filter(built, tmp_path):
    """Without promiscuous mode the pcap pktio passes only frames to its MAC
    02:00:00:00:00:02, broadcast and multicast (pcap.c:176-186)."""
    from odp_amd import pktgen as pg
    mine = pg.pad_to(pg.eth(dst=bytes.fromhex("020000000002")) + pg.ipv4() + pg.udp(), 60)
    other = pg.pad_to(pg.eth(dst=bytes.fromhex("020000000003")) + pg.ipv4() + pg.udp(), 60)
    bcast = pg.pad_to(pg.eth(dst=b"\xff" * 6) + pg.ipv4() + pg.udp(), 60)
    mcast = pg.pad_to(pg.eth(dst=bytes.fromhex("01005e000001")) + pg.ipv4() + pg.udp(), 60)
    p = str(tmp_path / "f.pcap")
    H.write_pcap(p, [mine, other, bcast, mcast])
    got, _, _ = H.run_driver(f"pcap:in={p}", None, "direct", layer=0, cls=0,
                             env={"RX_NO_PROMISC": "1"})
    assert _frames(got["pktin"]) == [mine, bcast, mcast]
    got, _, _ = H.run_driver(f"pcap:in={p}", None, "direct", layer=0, cls=0)
    assert _frames(got["pktin"]) == [mine, other, bcast, mcast]


@pytest.mark.parametrize("mode", ["direct", "sched", "queue"])
def test_loop_pktio_modes(built, mode):
    """Frames sent into the loop interface come back out of its input, in
    order, in every input mode."""
    got, st, _ = H.run_driver("loop", None, mode, layer=0, cls=0, src=UDP64)
    q = "pktin" if mode == "direct" else "odp-pktin-0-0"
    assert _frames(got[q]) == zoo.udp64_frames()


def test_rt_unit(built):
    """Pools, packets, queues, scheduler priorities / atomic ownership,
    aggregator vectors, cpumask, shm, time and helper parsers."""
    exe = os.path.join(H.ROOT, "tests", "_bin", "rt_unit")
    r = subprocess.run([exe], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stdout
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith(("ok ", "FAIL "))]
    assert lines and all(ln.startswith("ok ") for ln in lines), r.stdout


def test_example_classifier_links(built):
    """The reference's example/classifier source compiled unchanged against
    include/odp_api.h + include/odp/helper/odph_api.h (_build.build_example).
    Without a GPU it must stop at odp_pktio_start, loudly, not fall back to
    a CPU classifier."""
    if not os.path.exists(H.EXAMPLE):
        pytest.skip("example binary not built (reference tree absent at build time)")
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present: covered by tests/test_gpu_runtime.py")
    except ImportError:
        pass
    r = subprocess.run([H.EXAMPLE, "-t", "1", "-i", f"pcap:in={UDP64}", "-m", "0", "-p",
                        "ODP_PMR_SIP_ADDR:10.10.10.0:0xFFFFFF00:queue1", "-P", "-C",
                        "queue1:100", "-C", "DefaultCos:100"],
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=60,
                       cwd="/tmp")
    assert r.returncode != 0
    assert "GPU receive path unavailable" in r.stdout
    assert "CoSqueue1" in r.stdout   # the rules were configured through odp_cls_*
