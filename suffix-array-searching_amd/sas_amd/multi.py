"""One process, several GPUs: the C ABI's sas_build_multi / sas_search_multi
(include/sas.h).  REPLICATE cuts a batch into per-device query chunks
(the reference's rayon chunking, sst/bin/bench.rs:558-573); SHARD keeps part g of the
SA rank space on device g and routes every query to its part.  The torch.distributed
(one process per GPU) path is sas_amd.shard / bench.py --mode shard."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, lib
from .sa import _as_u8, _prefix_flags, _ptr, _quad_flags

MODES = {"replicate": _lib.SAS_MULTI_REPLICATE, "shard": _lib.SAS_MULTI_SHARD}


class SaMulti:
    def __init__(self, handle, n, devices, mode):
        self._h = handle
        self.n = n
        self.devices = list(devices)
        self.mode = mode

    @classmethod
    def build(cls, t, devices, mode: str = "replicate", lcp: bool = False, stree: bool = False,
              sector: bool = False, quad: bool | str = True, flags: int = 0,
              prefix: bool | int | None = None) -> "SaMulti":
        """t: host text (codes 0..3).  devices: device ordinals, repeats allowed.
        prefix: the prefix table for algo="prefix" (as SaNaive.build)."""
        t = np.ascontiguousarray(_as_u8(t))
        dv = np.ascontiguousarray(devices, np.int32)
        flags |= (_lib.SAS_BUILD_LCP if lcp else 0) | (_lib.SAS_BUILD_STREE if stree else 0)
        flags |= (_lib.SAS_BUILD_SECTOR if sector else 0) | _quad_flags(quad) | _prefix_flags(prefix, quad, len(t))
        h = C.c_void_p()
        check(lib().sas_build_multi(_ptr(t), len(t), _ptr(dv), len(dv), MODES[mode], flags, C.byref(h)))
        return cls(h, len(t), dv.tolist(), mode)

    def parts(self) -> int:
        return lib().sas_multi_parts(self._h)

    def stats(self, part: int) -> dict:
        st = _lib.SasStats()
        check(lib().sas_multi_get_stats(self._h, int(part), C.byref(st)))
        return st.as_dict()

    def search_batch(self, qbytes, qoff, qlen, algo: str = "quad") -> np.ndarray:
        """Ragged host queries, query k = qbytes[qoff[k] : qoff[k] + qlen[k]]; positions as
        sas_search_batch on one whole index."""
        qbytes = np.ascontiguousarray(_as_u8(qbytes))
        qoff = np.ascontiguousarray(qoff, np.uint64)
        qlen = np.ascontiguousarray(qlen, np.uint32)
        out = np.zeros(max(len(qoff), 1), np.uint64)
        check(lib().sas_search_multi(self._h, _ptr(qbytes), _ptr(qoff), _ptr(qlen), len(qoff), _lib.ALGOS[algo],
                                     _ptr(out), 0))
        return out[:len(qoff)]

    def free(self):
        if self._h:
            lib().sas_multi_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
