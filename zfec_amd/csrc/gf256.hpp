// gf256.hpp -- host-side GF(2^8) field and code-matrix construction.
//
// Everything here is O(k^3) per code or per decode call and stays on the host;
// the per-byte work is in kernels.hip.  Results are bit-identical to
// /root/reference/zfec/fec.c (pinned by tests/golden).
#pragma once
#include <cstddef>
#include <cstdint>

namespace zfec_hip {

struct Field {
    uint8_t exp[510];      // alpha^i, doubled (zfec/fec.c:28,140-142)
    int log[256];          // log[0] = 255 sentinel (zfec/fec.c:29,139)
    uint8_t inv[256];      // inv[0] = 0 (zfec/fec.c:30,149-152)
    uint8_t mul[256][256]; // (zfec/fec.c:58,77-86)
};

// Built once (std::call_once); replaces fec_init's generate_gf + _init_mul_table.
const Field& field();
bool field_ready();
void field_init();

inline uint8_t gf_mul(uint8_t a, uint8_t b) { return field().mul[a][b]; }

// zfec/fec.c:341-394: in-place inverse of a k x k Vandermonde matrix.
void invert_vandermonde(uint8_t* m, unsigned k);

// zfec/fec.c:430-479: systematic n x k encoding matrix.
void build_encoding_matrix(unsigned k, unsigned n, uint8_t* enc);

// zfec/fec.c:231-328: Gauss-Jordan inverse; false if singular.
bool invert_matrix(uint8_t* m, unsigned k);

// zfec/fec.c:512-525: decode matrix for received block numbers `index`.
bool build_decode_matrix(const uint8_t* enc, unsigned k, const unsigned* index, uint8_t* dec);

}  // namespace zfec_hip
