// shelfi_scheme.hpp — the reference's C++ plugin interface over the C ABI (header-only, C++17).
//
// Restates palisade_pybind/SHELFI_FHE/include/scheme.h:15-32 (abstract `Scheme`, 8 pure
// virtuals) and include/ckks.h:27-54 (`CKKS : Scheme`) for C++ callers such as the
// reference's smoke driver src/main.cpp:26-78, with PALISADE replaced by libshelfi
// (include/shelfi.h, HIP kernels on an MI355X).  Nothing here needs PALISADE or pybind11:
//
//   Scheme::loadCryptoParams()                 ckks.cpp:11-23  (prints on failure, never throws)
//   Scheme::genCryptoContextAndKeyGen()        ckks.cpp:25-59  (1 on success, 0 on a write error)
//   Scheme::encrypt_cpp(vector<double>)        ckks.cpp:107-167 -> the serialized batch
//   Scheme::computeWeightedAverage_cpp(vector<string>, vector<float>)
//                                              ckks.cpp:323-371 (size mismatch: prints, returns "")
//   Scheme::decrypt_cpp(string, unsigned long) ckks.cpp:217-260 -> n doubles
//
// The three pybind11-typed pure virtuals of scheme.h:24,26,28 (encrypt(py::array_t<double>)
// -> py::bytes, computeWeightedAverage(py::list, py::list) -> py::bytes, decrypt(string,
// unsigned long) -> py::array_t<double>) are declared too when pybind11 was included before
// this header (the extension module, fhe-fed_amd/pybind/binding.cpp), so the interface is
// scheme.h's exactly there and free of Python everywhere else.
//
// Errors: what PALISADE would throw surfaces as an exception — std::invalid_argument for
// bad arguments / out-of-range values (pybind11: ValueError), std::runtime_error otherwise
// (pybind11: RuntimeError); soft errors print as the reference does.  Byte format: the
// reference's own PALISADE cereal archives (ckks.cpp:98-100, :163-165) once keys are
// generated or loaded, or this library's blob (Options::wire_palisade = false; packed at the
// moduli's widths with Options::wire_packed); all are accepted as inputs.
#ifndef SHELFI_SCHEME_HPP_
#define SHELFI_SCHEME_HPP_

#include <cstdint>
#include <cstdlib>
#include <iostream>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "shelfi.h"

namespace shelfi {

// scheme.h:15-32
class Scheme {
 public:
  explicit Scheme(std::string scheme) : scheme_(std::move(scheme)) {}
  virtual ~Scheme() = default;

  virtual void loadCryptoParams() = 0;
  virtual int genCryptoContextAndKeyGen() = 0;
  virtual std::string encrypt_cpp(std::vector<double> learner_Data) = 0;
  virtual std::string computeWeightedAverage_cpp(std::vector<std::string> learners_Data,
                                                 std::vector<float> scalingFactors) = 0;
  virtual std::vector<double> decrypt_cpp(std::string learner_Data, unsigned long int data_dimensions) = 0;
#ifdef PYBIND11_VERSION_MAJOR
  virtual pybind11::bytes encrypt(pybind11::array_t<double> data_array) = 0;
  virtual pybind11::bytes computeWeightedAverage(pybind11::list learner_data, pybind11::list scaling_factors) = 0;
  virtual pybind11::array_t<double> decrypt(std::string learner_data, unsigned long int data_dimensions) = 0;
#endif

  const std::string& scheme() const { return scheme_; }

 private:
  std::string scheme_;
};

// Status code -> the exception PALISADE / pybind11 would give the caller.
inline void throw_on_error(int rc, const char* what) {
  if (rc == SHELFI_OK) return;
  const std::string msg = std::string(what) + ": " + shelfi_last_error();
  if (rc == SHELFI_ERR_ARG || rc == SHELFI_ERR_RANGE) throw std::invalid_argument(msg);
  throw std::runtime_error(msg);
}

// ckks.h:27-54.  The constructor is the reference's (scheme, batchSize, scaleFactorBits,
// cryptodir: ckks.cpp:5-9, multDepth 1 -> 2 RNS towers, ckks.cpp:26); Options are this
// library's extensions, defaulting to the reference's behaviour.
class CKKS : public Scheme {
 public:
  struct Options {
    unsigned multDepth = 1;     // towers = multDepth + 1 (the reference fixes 1)
    unsigned firstModBits = 60;
    unsigned ringDim = 0;       // 0: PALISADE's choice for the security level and batch
    int device = -1;            // HIP ordinal; -1: $LOCAL_RANK or 0 (one process per GPU)
    uint64_t seed = 0;          // deterministic encryption randomness (parity tests); 0: OS entropy
    bool decodeNoise = true;    // PALISADE 1.11's decode noise flooding (its Decrypt floods)
    bool wire_palisade = true;  // encrypt / aggregate answer in PALISADE's cereal archives
    bool wire_packed = false;   // with wire_palisade false: packed library blobs (version 2)
  };

  CKKS(std::string scheme, unsigned batchSize, unsigned scaleFactorBits, std::string cryptodir)
      : CKKS(std::move(scheme), batchSize, scaleFactorBits, std::move(cryptodir), Options{}) {}

  CKKS(std::string scheme, unsigned batchSize, unsigned scaleFactorBits, std::string cryptodir,
       const Options& opt)
      : Scheme(scheme), batchSize(batchSize), scaleFactorBits(scaleFactorBits), cryptodir(std::move(cryptodir)),
        opt_(opt) {
    if (scheme != "ckks" && scheme != "CKKS") throw std::invalid_argument("only the 'ckks' scheme is implemented");
    int dev = opt.device;
    if (dev < 0) {
      const char* lr = std::getenv("LOCAL_RANK");
      dev = lr ? std::atoi(lr) : 0;
    }
    throw_on_error(shelfi_ctx_create(opt.ringDim, opt.multDepth + 1, scaleFactorBits, opt.firstModBits, batchSize,
                                     dev, &ctx_),
                   "CKKS");
    try {
      if (opt.seed) throw_on_error(shelfi_set_seed(ctx_, opt.seed), "CKKS");
      if (!opt.decodeNoise) throw_on_error(shelfi_set_decode_noise(ctx_, 0, 1.0), "CKKS");
    } catch (...) {
      shelfi_ctx_destroy(ctx_);
      throw;
    }
  }
  ~CKKS() override { shelfi_ctx_destroy(ctx_); }
  CKKS(const CKKS&) = delete;
  CKKS& operator=(const CKKS&) = delete;

  // ckks.cpp:11-23: context, public and private key from cryptodir; a failure is printed
  // and the object stays usable for another load
  void loadCryptoParams() override {
    if (shelfi_load(ctx_, cryptodir.c_str()) != SHELFI_OK) {
      std::cerr << "Could not read serialization from " << cryptodir << "cryptocontext.txt: " << shelfi_last_error()
                << std::endl;
      return;
    }
    apply_wire_format();
  }

  // ckks.cpp:25-59: generate the context and keys and write them to cryptodir
  int genCryptoContextAndKeyGen() override {
    const int rc = shelfi_keygen(ctx_, cryptodir.c_str());
    if (rc == SHELFI_ERR_IO) {
      std::cerr << "Error writing serialization: " << shelfi_last_error() << std::endl;
      return 0;
    }
    throw_on_error(rc, "genCryptoContextAndKeyGen");
    apply_wire_format();
    return 1;
  }

  // ckks.cpp:107-167: ceil(n / batchSize) ciphertexts, serialized
  std::string encrypt_cpp(std::vector<double> learner_Data) override {
    size_t n = 0;
    throw_on_error(shelfi_encrypt_into(ctx_, learner_Data.data(), learner_Data.size(), nullptr, 0, &n), "encrypt");
    std::string out(n, '\0');
    throw_on_error(shelfi_encrypt_into(ctx_, learner_Data.data(), learner_Data.size(),
                                       reinterpret_cast<uint8_t*>(&out[0]), out.size(), &n),
                   "encrypt");
    return out;
  }

  // ckks.cpp:323-371: sum_i EvalMult(ct_i, (float)w_i), EvalAdd; weights are float already
  std::string computeWeightedAverage_cpp(std::vector<std::string> learners_Data,
                                         std::vector<float> scalingFactors) override {
    if (learners_Data.size() != scalingFactors.size()) {
      std::cout << "Error: learners_Data and scalingFactors size mismatch" << std::endl;
      return "";
    }
    const size_t C = learners_Data.size();
    std::vector<const uint8_t*> ptr(C);
    std::vector<size_t> len(C);
    for (size_t i = 0; i < C; ++i) {
      ptr[i] = reinterpret_cast<const uint8_t*>(learners_Data[i].data());
      len[i] = learners_Data[i].size();
    }
    size_t n = 0;
    throw_on_error(shelfi_weighted_average_into(ctx_, ptr.data(), len.data(), scalingFactors.data(), C, nullptr, 0, &n),
                   "computeWeightedAverage");
    std::string out(n, '\0');
    throw_on_error(shelfi_weighted_average_into(ctx_, ptr.data(), len.data(), scalingFactors.data(), C,
                                                reinterpret_cast<uint8_t*>(&out[0]), out.size(), &n),
                   "computeWeightedAverage");
    return out;
  }

  // ckks.cpp:217-260: the first data_dimensions decoded slots of the batch
  std::vector<double> decrypt_cpp(std::string learner_Data, unsigned long int data_dimensions) override {
    std::vector<double> out(data_dimensions);
    throw_on_error(shelfi_decrypt(ctx_, reinterpret_cast<const uint8_t*>(learner_Data.data()), learner_Data.size(),
                                  data_dimensions, out.data()),
                   "decrypt");
    return out;
  }

#ifdef PYBIND11_VERSION_MAJOR
  // scheme.h:24,26,28, as binding.cpp:26-31 exposes them (the GIL is released around the
  // device work, which the reference never does)
  pybind11::bytes encrypt(pybind11::array_t<double> data_array) override {
    pybind11::array_t<double, pybind11::array::c_style | pybind11::array::forcecast> a(data_array);
    std::vector<double> v(a.data(), a.data() + a.size());
    std::string s;
    {
      pybind11::gil_scoped_release nogil;
      s = encrypt_cpp(std::move(v));
    }
    return pybind11::bytes(s);
  }
  pybind11::bytes computeWeightedAverage(pybind11::list learner_data, pybind11::list scaling_factors) override {
    if (learner_data.size() != scaling_factors.size()) {
      std::cout << "Error: learner_data and scaling_factors size mismatch" << std::endl;
      return pybind11::bytes("");
    }
    std::vector<std::string> d;
    std::vector<float> w;
    for (size_t i = 0; i < learner_data.size(); ++i) {
      d.push_back(learner_data[i].cast<std::string>());  // ckks.cpp:276 (raw bytes via py::str)
      w.push_back(scaling_factors[i].cast<float>());     // ckks.cpp:287 narrows to float
    }
    std::string s;
    {
      pybind11::gil_scoped_release nogil;
      s = computeWeightedAverage_cpp(std::move(d), std::move(w));
    }
    return pybind11::bytes(s);
  }
  pybind11::array_t<double> decrypt(std::string learner_data, unsigned long int data_dimensions) override {
    std::vector<double> v;
    {
      pybind11::gil_scoped_release nogil;
      v = decrypt_cpp(std::move(learner_data), data_dimensions);
    }
    return pybind11::array_t<double>((pybind11::ssize_t)v.size(), v.data());
  }
#endif

  // ckks.h:31-33 state, read-only here (cc / pk / sk live in the library context)
  unsigned getBatchSize() const { return batchSize; }
  unsigned getScaleFactorBits() const { return scaleFactorBits; }
  const std::string& getCryptodir() const { return cryptodir; }
  shelfi_ctx* context() const { return ctx_; }

 private:
  // keys generated here or loaded from PALISADE files carry the context object and key tag
  // PALISADE's archive format needs
  void apply_wire_format() {
    throw_on_error(shelfi_set_wire_format(ctx_, opt_.wire_palisade ? 1 : opt_.wire_packed ? 2 : 0), "wire format");
  }

  unsigned batchSize;
  unsigned scaleFactorBits;
  std::string cryptodir;
  Options opt_;
  shelfi_ctx* ctx_ = nullptr;
};

}  // namespace shelfi

#endif  // SHELFI_SCHEME_HPP_
