// palisade_io.h — reader for PALISADE 1.11 cereal-binary context/key files.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace shelfi {

struct PalisadeContext {
  uint32_t N = 0;
  std::vector<uint64_t> q, psi;
};

// cryptocontext.txt written by ckks.cpp:41 (Serial::SerializeToFile, SerType::BINARY)
PalisadeContext palisade_read_context(const std::string& bytes);
// key-public.txt / key-private.txt written by ckks.cpp:48,53 -> pk [2][L][N], sk [L][N]
void palisade_read_keys(const std::string& pub, const std::string& priv, uint32_t N,
                        const std::vector<uint64_t>& q, std::vector<uint64_t>& pk,
                        std::vector<uint64_t>& sk);

}  // namespace shelfi
