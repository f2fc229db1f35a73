"""The C++ host API (include/sas.hpp, the reference's Rust names over the C ABI) through
tests/cpp/test_api.cpp: it compiles against the headers and links libsas_amd.so on the CPU,
and on the GPU it passes the reference-shaped checks (sst/src/test.rs differential + KAT,
binary_search / binary_search_batch / interpolation_search positions and cnt against the
oracle, search_prefix against a text scan, the panic on bad input)."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(REPO, "tests", "cpp")


def test_header_compiles_standalone(tmp_path):
    src = tmp_path / "t.cpp"
    src.write_text('#include "sas.hpp"\nint main() { return sizeof(sas::SaNaive) > 0 ? 0 : 1; }\n')
    subprocess.check_call(["g++", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-fsyntax-only",
                           "-I", os.path.join(REPO, "include"), str(src)])


def test_cpp_api_links():
    subprocess.check_call(["make", "-s", "-C", CPP])
    assert os.access(os.path.join(CPP, "test_api"), os.X_OK)


@pytest.mark.gpu
def test_cpp_api_on_gpu():
    exe = os.path.join(CPP, "test_api")
    assert os.path.exists(exe), "build() compiles tests/cpp/test_api"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "cpp api ok" in r.stdout
