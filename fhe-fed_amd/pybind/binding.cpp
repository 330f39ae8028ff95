// INTEGRATION.md Option B, built: a pybind11 extension module named SHELFI_FHE whose
// classes and method table are the reference's (palisade_pybind/SHELFI_FHE/src/
// binding.cpp:14-31: Scheme, CKKS(scheme, batchSize, scaleFactorBits, cryptodir) with
// loadCryptoParams / genCryptoContextAndKeyGen / encrypt / decrypt /
// computeWeightedAverage and the *_cpp aliases), implemented by the C++ plugin classes
// of include/shelfi_scheme.hpp (scheme.h's Scheme, ckks.h's CKKS) over the C ABI
// (include/shelfi.h) instead of PALISADE.  A caller that imports this .so in place of the
// reference's module sees the same names, defaults, argument conversions and soft errors
// (ckks.cpp:11-23 prints on a failed load; ckks.cpp:265-268 prints and returns b"" on a
// weight / learner count mismatch).  No torch, no Python-side wrapper.
//
// Like the reference module, encrypt answers in PALISADE's own wire format (a cereal
// archive of vector<Ciphertext<DCRTPoly>>, ckks.cpp:98-100) once keys are generated or
// loaded; keyword-only extras (multDepth, seed, decodeNoise, wireFormat, device) are the
// ctypes mirror's (fhe-fed_amd/SHELFI_FHE/__init__.py) and default to the reference's
// behaviour.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <cstring>
#include <iostream>
#include <memory>
#include <string>
#include <vector>

// after pybind11: Scheme then carries scheme.h's three py-typed pure virtuals as well
#include "shelfi_scheme.hpp"

namespace py = pybind11;
using shelfi::CKKS;
using shelfi::Scheme;

namespace {

// CKKS(scheme, batchSize, scaleFactorBits, cryptodir, *, extras) -> the C++ plugin object
std::unique_ptr<CKKS> make_ckks(const std::string& scheme, unsigned batchSize, unsigned scaleFactorBits,
                                const std::string& cryptodir, unsigned multDepth, uint64_t seed, bool decodeNoise,
                                const std::string& wireFormat, int device) {
  if (wireFormat != "palisade" && wireFormat != "shelfi" && wireFormat != "packed")
    throw py::value_error("wireFormat must be 'palisade', 'shelfi' or 'packed'");
  CKKS::Options o;
  o.multDepth = multDepth;
  o.seed = seed;
  o.decodeNoise = decodeNoise;
  o.wire_palisade = wireFormat == "palisade";
  o.wire_packed = wireFormat == "packed";
  o.device = device;
  return std::make_unique<CKKS>(scheme, batchSize, scaleFactorBits, cryptodir, o);
}

// binding.cpp:27,29,31 register the *_cpp names on the py-typed methods; here they go
// through the C++ interface's *_cpp virtuals (Scheme's vtable) and return the same Python
// types the reference's aliases do.
py::bytes encrypt_cpp(Scheme& s, py::array_t<double, py::array::c_style | py::array::forcecast> a) {
  std::vector<double> v((size_t)a.size());
  if (a.size()) std::memcpy(v.data(), a.data(), sizeof(double) * (size_t)a.size());
  std::string out;
  {
    py::gil_scoped_release nogil;
    out = s.encrypt_cpp(std::move(v));
  }
  return py::bytes(out);
}

py::bytes wavg_cpp(Scheme& s, py::list learner_data, py::list scaling_factors) {
  if (learner_data.size() != scaling_factors.size()) {
    std::cout << "Error: learner_data and scaling_factors size mismatch" << std::endl;
    return py::bytes("");
  }
  std::vector<std::string> d;
  std::vector<float> w;
  for (size_t i = 0; i < learner_data.size(); ++i) {
    d.push_back(learner_data[i].cast<std::string>());
    w.push_back(scaling_factors[i].cast<float>());
  }
  std::string out;
  {
    py::gil_scoped_release nogil;
    out = s.computeWeightedAverage_cpp(std::move(d), std::move(w));
  }
  return py::bytes(out);
}

py::array_t<double> decrypt_cpp(Scheme& s, std::string data, unsigned long n) {
  std::vector<double> v;
  {
    py::gil_scoped_release nogil;
    v = s.decrypt_cpp(std::move(data), n);
  }
  return py::array_t<double>((py::ssize_t)v.size(), v.data());
}

}  // namespace

PYBIND11_MODULE(SHELFI_FHE, mod) {
  mod.doc() = "MI355X CKKS weighted-average aggregator: the SHELFI_FHE module's classes over libshelfi";
  py::class_<Scheme>(mod, "Scheme");
  py::class_<CKKS, Scheme>(mod, "CKKS")
      .def(py::init(&make_ckks), py::arg("scheme") = std::string("ckks"), py::arg("batchSize") = 4096u,
           py::arg("scaleFactorBits") = 52u, py::arg("cryptodir") = std::string("../resources/cryptoparams/"),
           py::kw_only(), py::arg("multDepth") = 1u, py::arg("seed") = (uint64_t)0,
           py::arg("decodeNoise") = true, py::arg("wireFormat") = std::string("palisade"),
           py::arg("device") = -1)
      .def("loadCryptoParams", &CKKS::loadCryptoParams)
      .def("genCryptoContextAndKeyGen", &CKKS::genCryptoContextAndKeyGen)
      .def("encrypt", &CKKS::encrypt)
      .def("encrypt_cpp", &encrypt_cpp)
      .def("decrypt", &CKKS::decrypt)
      .def("decrypt_cpp", &decrypt_cpp)
      .def("computeWeightedAverage", &CKKS::computeWeightedAverage)
      .def("computeWeightedAverage_cpp", &wavg_cpp);
  mod.attr("__version__") = "dev";
}
