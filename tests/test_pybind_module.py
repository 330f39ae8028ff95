"""CPU checks of the native pybind11 module (INTEGRATION.md Option B): it loads against
libshelfi.so, carries the reference module's classes, method table and constructor
defaults (palisade_pybind/SHELFI_FHE/src/binding.cpp:14-31), and constructing a CKKS
without a HIP device fails loudly instead of falling back to anything."""
import inspect

import pytest

import pybind_native

METHODS = ["loadCryptoParams", "genCryptoContextAndKeyGen", "encrypt", "encrypt_cpp", "decrypt",
           "decrypt_cpp", "computeWeightedAverage", "computeWeightedAverage_cpp"]


@pytest.fixture(scope="module")
def nm():
    return pybind_native.load()


def test_classes_and_method_table(nm):
    assert issubclass(nm.CKKS, nm.Scheme)
    for name in METHODS:
        assert callable(getattr(nm.CKKS, name)), name


def test_constructor_defaults_are_the_references(nm):
    doc = nm.CKKS.__init__.__doc__
    for frag in ("scheme: str = 'ckks'", "= 4096", "= 52", "cryptodir: str = '../resources/cryptoparams/'",
                 "wireFormat: str = 'palisade'", "multDepth"):
        assert frag in doc, (frag, doc)


def test_decrypt_and_wavg_signatures(nm):
    # ckks.h:45-51: encrypt(array_t<double>) -> bytes, computeWeightedAverage(list, list)
    # -> bytes, decrypt(string, unsigned long) -> array_t<double>
    assert "numpy.float64]) -> bytes" in nm.CKKS.encrypt.__doc__
    assert "arg0: list, arg1: list) -> bytes" in nm.CKKS.computeWeightedAverage.__doc__
    d = nm.CKKS.decrypt.__doc__
    assert "arg0: str, arg1:" in d and "numpy.float64]" in d


def test_no_device_is_a_loud_error(nm):
    try:
        nm.CKKS()
    except RuntimeError as e:
        assert "no HIP device" in str(e)
    else:
        pytest.skip("a device is present (tests/test_gpu_pybind_module.py covers it)")


def test_argument_errors_before_the_device(nm):
    with pytest.raises(ValueError, match="wireFormat"):
        nm.CKKS(wireFormat="protobuf")
    with pytest.raises(ValueError, match="scheme"):
        nm.CKKS("bfv")
    with pytest.raises(TypeError):
        nm.CKKS("ckks", 4096, 52, "x", 3)  # the extras are keyword-only
    assert inspect.isclass(nm.CKKS)
