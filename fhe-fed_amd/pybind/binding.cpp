// INTEGRATION.md Option B, built: a pybind11 extension module named SHELFI_FHE whose
// classes and method table are the reference's (palisade_pybind/SHELFI_FHE/src/
// binding.cpp:14-31: Scheme, CKKS(scheme, batchSize, scaleFactorBits, cryptodir) with
// loadCryptoParams / genCryptoContextAndKeyGen / encrypt / decrypt /
// computeWeightedAverage and the *_cpp aliases), implemented over the C ABI
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

#include <cstdint>
#include <cstdlib>
#include <iostream>
#include <stdexcept>
#include <string>
#include <vector>

#include "shelfi.h"

namespace py = pybind11;

namespace {

void raise(int rc, const char* what) {
  if (rc == SHELFI_OK) return;
  const std::string msg = std::string(what) + ": " + shelfi_last_error();
  if (rc == SHELFI_ERR_ARG || rc == SHELFI_ERR_RANGE) throw py::value_error(msg);
  throw std::runtime_error(msg);
}

// library-owned output -> Python bytes
py::bytes take(uint8_t* p, size_t n) {
  py::bytes b(reinterpret_cast<const char*>(p), n);
  shelfi_free(p);
  return b;
}

}  // namespace

// scheme.h:15-32: the base holds the scheme name only
class Scheme {
 public:
  explicit Scheme(std::string name) : scheme_(std::move(name)) {}
  virtual ~Scheme() = default;
  const std::string& scheme() const { return scheme_; }

 private:
  std::string scheme_;
};

// ckks.h:27-54 over shelfi_ctx: multDepth 1 (ckks.cpp:26) -> 2 towers, 60-bit first modulus
class CKKS : public Scheme {
 public:
  CKKS(std::string& scheme, unsigned batchSize, unsigned scaleFactorBits, std::string& cryptodir,
       unsigned multDepth, uint64_t seed, bool decodeNoise, const std::string& wireFormat, int device)
      : Scheme(scheme), dir_(cryptodir) {
    if (scheme != "ckks" && scheme != "CKKS") throw py::value_error("only the 'ckks' scheme is implemented");
    if (wireFormat != "palisade" && wireFormat != "shelfi")
      throw py::value_error("wireFormat must be 'palisade' or 'shelfi'");
    palisade_wire_ = wireFormat == "palisade";
    if (device < 0) {  // one process per GPU: LOCAL_RANK picks the card, as in the ctypes mirror
      const char* lr = std::getenv("LOCAL_RANK");
      device = lr ? std::atoi(lr) : 0;
    }
    raise(shelfi_ctx_create(0, multDepth + 1, scaleFactorBits, 60, batchSize, device, &ctx_), "CKKS");
    if (seed) raise(shelfi_set_seed(ctx_, seed), "CKKS");
    if (!decodeNoise) raise(shelfi_set_decode_noise(ctx_, 0, 1.0), "CKKS");
  }
  ~CKKS() override { shelfi_ctx_destroy(ctx_); }
  CKKS(const CKKS&) = delete;
  CKKS& operator=(const CKKS&) = delete;

  void loadCryptoParams() {  // ckks.cpp:11-23: failures are printed, not raised
    if (shelfi_load(ctx_, dir_.c_str()) != SHELFI_OK)
      std::cerr << "Could not load the crypto parameters from " << dir_ << ": " << shelfi_last_error()
                << std::endl;
    else
      wire();
  }

  int genCryptoContextAndKeyGen() {  // ckks.cpp:25-59
    const int rc = shelfi_keygen(ctx_, dir_.c_str());
    if (rc != SHELFI_OK) {
      std::cerr << shelfi_last_error() << std::endl;
      return 0;
    }
    wire();
    return 1;
  }

  py::bytes encrypt(py::array_t<double, py::array::c_style | py::array::forcecast> values) {  // :61-104
    uint8_t* out = nullptr;
    size_t len = 0;
    int rc;
    {
      py::gil_scoped_release nogil;
      rc = shelfi_encrypt(ctx_, values.data(), (size_t)values.size(), &out, &len);
    }
    raise(rc, "encrypt");
    return take(out, len);
  }

  py::array_t<double> decrypt(const std::string& data, unsigned long n) {  // :170-213
    py::array_t<double> out((py::ssize_t)n);
    double* dst = out.mutable_data();
    int rc;
    {
      py::gil_scoped_release nogil;
      rc = shelfi_decrypt(ctx_, reinterpret_cast<const uint8_t*>(data.data()), data.size(), n, dst);
    }
    raise(rc, "decrypt");
    return out;
  }

  py::bytes computeWeightedAverage(py::list learner_data, py::list scaling_factors) {  // :264-320
    if (learner_data.size() != scaling_factors.size()) {
      std::cout << "Error: learner_data and scaling_factors size mismatch" << std::endl;
      return py::bytes("");
    }
    const size_t C = learner_data.size();
    std::vector<std::string> keep;  // the uploads, held for the call
    keep.reserve(C);
    std::vector<float> w;
    w.reserve(C);
    for (size_t i = 0; i < C; ++i) {
      keep.push_back(learner_data[i].cast<std::string>());
      w.push_back(scaling_factors[i].cast<float>());  // ckks.cpp:287 narrows to float
    }
    std::vector<const uint8_t*> ptr(C);
    std::vector<size_t> len(C);
    for (size_t i = 0; i < C; ++i) {
      ptr[i] = reinterpret_cast<const uint8_t*>(keep[i].data());
      len[i] = keep[i].size();
    }
    uint8_t* out = nullptr;
    size_t n = 0;
    int rc;
    {
      py::gil_scoped_release nogil;
      rc = shelfi_weighted_average(ctx_, ptr.data(), len.data(), w.data(), C, &out, &n);
    }
    raise(rc, "computeWeightedAverage");
    return take(out, n);
  }

 private:
  // keys generated here or loaded from PALISADE files carry the context object and key
  // tag the archive format needs
  void wire() { raise(shelfi_set_wire_format(ctx_, palisade_wire_ ? 1 : 0), "wire format"); }

  std::string dir_;
  bool palisade_wire_ = true;
  shelfi_ctx* ctx_ = nullptr;
};

PYBIND11_MODULE(SHELFI_FHE, mod) {
  mod.doc() = "MI355X CKKS weighted-average aggregator: the SHELFI_FHE module's classes over libshelfi";
  py::class_<Scheme>(mod, "Scheme");
  py::class_<CKKS, Scheme>(mod, "CKKS")
      .def(py::init<std::string&, unsigned, unsigned, std::string&, unsigned, uint64_t, bool,
                    const std::string&, int>(),
           py::arg("scheme") = std::string("ckks"), py::arg("batchSize") = 4096u,
           py::arg("scaleFactorBits") = 52u, py::arg("cryptodir") = std::string("../resources/cryptoparams/"),
           py::kw_only(), py::arg("multDepth") = 1u, py::arg("seed") = (uint64_t)0,
           py::arg("decodeNoise") = true, py::arg("wireFormat") = std::string("palisade"),
           py::arg("device") = -1)
      .def("loadCryptoParams", &CKKS::loadCryptoParams)
      .def("genCryptoContextAndKeyGen", &CKKS::genCryptoContextAndKeyGen)
      .def("encrypt", &CKKS::encrypt)
      .def("encrypt_cpp", &CKKS::encrypt)
      .def("decrypt", &CKKS::decrypt)
      .def("decrypt_cpp", &CKKS::decrypt)
      .def("computeWeightedAverage", &CKKS::computeWeightedAverage)
      .def("computeWeightedAverage_cpp", &CKKS::computeWeightedAverage);
  mod.attr("__version__") = "dev";
}
