"""odp_amd -- MI355X-native drop-in for OpenDataPlane linux-generic's packet
parse + PMR classifier receive path.

  include/mi_cls.h        C ABI of the gfx950 HIP kernels (libmi_cls.so)
  include/odp_cls_api.h   ODP classification API surface (libodp_cls.so, C)
  odp_amd.cls             ctypes mirror of that API (tests, bench)
  odp_amd.pktgen          packet construction / synthetic batches
  odp_amd.rules           rule programs and the BASELINE.json workloads
"""
__all__ = ["cls", "pktgen", "rules"]
