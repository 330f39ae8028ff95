"""The reference's C++ plugin interface (include/scheme.h:15-32, include/ckks.h:27-54) restated
by include/shelfi_scheme.hpp, and its smoke driver (src/main.cpp:26-78) restated by
fhe-fed_amd/csrc/cpp_client.cpp.

CPU: the header compiles as C++17 without pybind11 (and with it, carrying scheme.h's eight
pure virtuals), `CKKS` is a concrete `Scheme`, and the client fails loudly without a device.
GPU: the client runs main.cpp's flow — 100 values U[0,100) from a default-seeded
std::default_random_engine, three copies of one encryption, weights 0.5/0.3/0.5 — through
the abstract interface on the reference's own PALISADE keys; its archives hold exactly the
oracle's encryption and aggregate, and the decryption is within 1e-7 of 1.3 x.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import PALISADE_DIR, ROOT

CLIENT = os.path.join(ROOT, "fhe-fed_amd", "SHELFI_FHE", "shelfi_cpp_client")
INC = os.path.join(ROOT, "include")


def _ensure_client():
    if not os.path.exists(CLIENT):
        subprocess.run(["make", "-C", os.path.join(ROOT, "fhe-fed_amd", "csrc"), "../SHELFI_FHE/shelfi_cpp_client"],
                       check=True, capture_output=True, timeout=600)
    return CLIENT


ABSTRACT_CHECK = r"""
#include <type_traits>
#include "shelfi_scheme.hpp"
static_assert(std::is_abstract<shelfi::Scheme>::value, "Scheme is the abstract plugin interface");
static_assert(!std::is_abstract<shelfi::CKKS>::value, "CKKS implements every pure virtual");
static_assert(std::is_base_of<shelfi::Scheme, shelfi::CKKS>::value, "CKKS : Scheme");
static_assert(std::has_virtual_destructor<shelfi::Scheme>::value, "virtual ~Scheme");
// scheme.h:23-31 signatures
using S = shelfi::Scheme;
static_assert(std::is_same<decltype(&S::encrypt_cpp), std::string (S::*)(std::vector<double>)>::value, "");
static_assert(std::is_same<decltype(&S::computeWeightedAverage_cpp),
              std::string (S::*)(std::vector<std::string>, std::vector<float>)>::value, "");
static_assert(std::is_same<decltype(&S::decrypt_cpp),
              std::vector<double> (S::*)(std::string, unsigned long int)>::value, "");
static_assert(std::is_same<decltype(&S::loadCryptoParams), void (S::*)()>::value, "");
static_assert(std::is_same<decltype(&S::genCryptoContextAndKeyGen), int (S::*)()>::value, "");
#ifdef PYBIND11_VERSION_MAJOR
static_assert(std::is_same<decltype(&S::encrypt), pybind11::bytes (S::*)(pybind11::array_t<double>)>::value, "");
static_assert(std::is_same<decltype(&S::computeWeightedAverage),
              pybind11::bytes (S::*)(pybind11::list, pybind11::list)>::value, "");
static_assert(std::is_same<decltype(&S::decrypt),
              pybind11::array_t<double> (S::*)(std::string, unsigned long int)>::value, "");
#endif
int main() { return 0; }
"""


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
@pytest.mark.parametrize("with_pybind", [False, True])
def test_interface_is_schemes(tmp_path, with_pybind):
    src = tmp_path / "check.cpp"
    pre = "#include <pybind11/pybind11.h>\n#include <pybind11/numpy.h>\n" if with_pybind else ""
    src.write_text(pre + ABSTRACT_CHECK)
    cmd = ["g++", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-fsyntax-only", "-I" + INC, str(src)]
    if with_pybind:
        import sysconfig

        pybind11 = pytest.importorskip("pybind11")
        cmd[1:1] = ["-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"]]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr


def test_cpp_client_fails_loudly_without_device():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present: test_cpp_client_runs_main_cpp_flow runs instead")
    p = subprocess.run([_ensure_client(), PALISADE_DIR], capture_output=True, text=True, timeout=60)
    assert p.returncode == 1
    assert "no HIP device" in p.stderr


@pytest.mark.gpu
def test_cpp_client_runs_main_cpp_flow(tmp_path):
    import oracle as O
    import palisade_fixture as P
    import SHELFI_FHE as m

    out = str(tmp_path) + os.sep
    p = subprocess.run([_ensure_client(), PALISADE_DIR, out, "42"], capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "Computing 0.5*L + 0.3*L + 0.5*L" in p.stdout and "Result:" in p.stdout
    x = np.fromfile(out + "input.f64", np.float64)
    assert x.size == 100 and (x >= 0).all() and (x < 100).all()
    ctx, pk, sk = P.read_keys(PALISADE_DIR)
    q, psi = np.array(ctx["q"], np.uint64), np.array(ctx["psi"], np.uint64)
    N, S = 8192, 4096
    delta = float(q[-1])
    enc_info, enc = m.palisade_parse(open(out + "encrypted.bin", "rb").read())
    assert enc_info["num_cts"] == 1 and enc_info["vector_archive"]
    assert np.array_equal(enc, O.encrypt_vector(x, pk, q, psi, N, S, delta, seed=42, g0=0))
    agg_info, agg = m.palisade_parse(open(out + "aggregate.bin", "rb").read())
    assert agg_info["depth"] == 2
    w = [0.5, 0.3, 0.5]
    assert np.array_equal(agg, O.wavg([enc, enc, enc], w, q, delta))
    got = np.fromfile(out + "decrypted.f64", np.float64)
    assert np.array_equal(got, O.decrypt_vector(agg, sk, q, psi, S, delta * delta, 100))
    exp = sum(float(np.float32(wi)) for wi in w) * x
    assert np.abs(got - exp).max() < 1e-7
