"""The drop-in boundary from plain C (fhe-fed_amd/csrc/c_client.c, no Python in the
loop): the header compiles as strict C99, the client links against libshelfi.so, fails
loudly without a gfx950 device (CPU), and on an MI355X runs keygen (PALISADE files) ->
load in a second context -> encrypt (blob and PALISADE wire) -> weighted average ->
decrypt (exact and flooded) plus the error paths (GPU)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

CLIENT = os.path.join(ROOT, "fhe-fed_amd", "SHELFI_FHE", "shelfi_c_client")
SRC = os.path.join(ROOT, "fhe-fed_amd", "csrc", "c_client.c")


def _ensure_client():
    if not os.path.exists(CLIENT):  # normally built by build() / make next to libshelfi.so
        subprocess.run(["make", "-C", os.path.join(ROOT, "fhe-fed_amd", "csrc"),
                        "../SHELFI_FHE/shelfi_c_client"], check=True, capture_output=True, timeout=600)
    return CLIENT


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_header_is_strict_c99():
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-pedantic", "-fsyntax-only", SRC],
                   check=True, capture_output=True, timeout=60)


def test_client_fails_loudly_without_device():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present: tests/test_c_client.py::test_c_client_round_trips runs instead")
    p = subprocess.run([_ensure_client(), "/tmp/shelfi_c_client_nogpu"], capture_output=True, text=True,
                       timeout=60)
    assert p.returncode == 1
    assert "-2" in p.stderr and "gfx950" in p.stderr  # SHELFI_ERR_DEVICE and its message


@pytest.mark.gpu
def test_c_client_round_trips(tmp_path):
    p = subprocess.run([_ensure_client(), str(tmp_path)], capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "C CLIENT OK" in p.stdout
    for f in ("cryptocontext.txt", "key-public.txt", "key-private.txt"):
        assert (tmp_path / f).stat().st_size > 0
