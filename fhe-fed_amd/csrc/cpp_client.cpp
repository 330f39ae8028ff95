// cpp_client.cpp — the reference's C++ smoke driver (palisade_pybind/SHELFI_FHE/src/main.cpp:26-78)
// written against this library's C++ plugin interface (include/shelfi_scheme.hpp): the same
// flow through the abstract Scheme's *_cpp virtuals, no PALISADE, no pybind11.
//
//   CKKS("ckks", 4096, 52, cryptodir); loadCryptoParams()            main.cpp:31-36
//   100 values U[0,100) from a default-seeded std::default_random_engine   main.cpp:8-23,41
//   encrypt_cpp -> three copies -> computeWeightedAverage_cpp(0.5, 0.3, 0.5)  main.cpp:48-67
//   decrypt_cpp(result, 100) and print                               main.cpp:73-78
//
// usage: shelfi_cpp_client <cryptodir/> [outdir/ [seed]]
// With outdir, the inputs, the encrypted batch, the aggregate and the decryption are written
// there for tests/test_gpu_cpp_client.py to check against the oracle; seed != 0 makes the
// encryption randomness reproducible (CKKS::Options::seed) and turns decode flooding off.
#include <fstream>
#include <iostream>
#include <random>
#include <string>
#include <vector>

#include "shelfi_scheme.hpp"

using namespace std;

static void generateRandomData(vector<double>& learner_Data, int rows) {
  uniform_real_distribution<double> unif(0, 100);
  default_random_engine re;
  for (int i = 0; i < rows; i++) learner_Data.push_back(unif(re));
}

static void write_file(const string& path, const void* p, size_t n) {
  ofstream f(path, ios::binary);
  f.write(static_cast<const char*>(p), (streamsize)n);
  if (!f) throw runtime_error("cannot write " + path);
}

static ostream& operator<<(ostream& os, const vector<double>& v) {
  os << "[";
  for (size_t i = 0; i < v.size(); ++i) os << (i ? ", " : "") << v[i];
  return os << "]";
}

int main(int argc, char** argv) {
  if (argc < 2) {
    cerr << "usage: " << argv[0] << " <cryptodir/> [outdir/ [seed]]" << endl;
    return 2;
  }
  const string cryptodir = argv[1];
  const string outdir = argc > 2 ? argv[2] : "";
  shelfi::CKKS::Options opt;
  if (argc > 3) {
    opt.seed = stoull(argv[3]);
    opt.decodeNoise = opt.seed == 0;
  }
  try {
    // the plugin is used through its abstract interface, as the reference's Scheme is
    shelfi::CKKS ckks("ckks", 4096, 52, cryptodir, opt);
    shelfi::Scheme& fhe_helper = ckks;
    fhe_helper.loadCryptoParams();

    vector<double> learner_Data;
    generateRandomData(learner_Data, 100);
    cout << "Learner Data: " << endl << learner_Data << endl << endl;

    cout << "Encrypting" << endl;
    string enc_result = fhe_helper.encrypt_cpp(learner_Data);

    vector<string> learners_Data{enc_result, enc_result, enc_result};
    vector<float> scalingFactors{0.5f, 0.3f, 0.5f};
    cout << "Computing 0.5*L + 0.3*L + 0.5*L" << endl;
    string pwa_result = fhe_helper.computeWeightedAverage_cpp(learners_Data, scalingFactors);

    const unsigned long int data_dimensions = learner_Data.size();
    cout << "Decrypting" << endl;
    vector<double> pwa_res_pt = fhe_helper.decrypt_cpp(pwa_result, data_dimensions);
    cout << "Result:" << endl << pwa_res_pt << endl;

    if (!outdir.empty()) {
      write_file(outdir + "input.f64", learner_Data.data(), learner_Data.size() * 8);
      write_file(outdir + "encrypted.bin", enc_result.data(), enc_result.size());
      write_file(outdir + "aggregate.bin", pwa_result.data(), pwa_result.size());
      write_file(outdir + "decrypted.f64", pwa_res_pt.data(), pwa_res_pt.size() * 8);
    }
    // the interface's soft error: a size mismatch prints and answers "" (ckks.cpp:325-328)
    if (!fhe_helper.computeWeightedAverage_cpp(learners_Data, {0.5f}).empty()) return 1;
  } catch (const exception& e) {
    cerr << "error: " << e.what() << endl;
    return 1;
  }
  return 0;
}
