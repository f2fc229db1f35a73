"""The u32 layouts' host builders on the CPU (no GPU): tests/cpp/sst_host_check.cpp builds
every PartitionedSTree16 marker (Simple, Compact, L1, Overlapping, Map) with the library's
own builder code (csrc/sst_host.hpp) at the sizes of sst/test.rs:146-153 and the b of
:222-254, walks each with the search kernels' index arithmetic, and compares every answer
with SortedVec::binary_search (sst/binary_search.rs:37-49)."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tests", "cpp", "sst_host_check.cpp")


def test_partitioned_builders_cpu(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    exe = tmp_path / "sst_host_check"
    subprocess.run([hipcc, "-O2", "-std=c++17", SRC, "-o", str(exe)], check=True, capture_output=True, timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "sst host ok" in r.stdout
