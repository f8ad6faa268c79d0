// gf256.cpp -- host GF(2^8) arithmetic and code matrices (see gf256.hpp).
#include "gf256.hpp"

#include <atomic>
#include <cstring>
#include <mutex>
#include <utility>
#include <vector>

namespace zfec_hip {

namespace {
Field g_field;
std::once_flag g_once;
std::atomic<bool> g_ready{false};  // read by fec_new on any thread

// Reduction polynomial x^8+x^4+x^3+x^2+1; zfec/fec.c:16 writes it as the
// coefficient string "101110001".
constexpr unsigned kPoly = 0x11D;

void build_field() {
    Field& f = g_field;
    unsigned x = 1;
    for (int i = 0; i < 255; ++i) {
        f.exp[i] = static_cast<uint8_t>(x);
        f.exp[i + 255] = static_cast<uint8_t>(x);
        f.log[x] = i;
        x <<= 1;
        if (x & 0x100) x ^= kPoly;
    }
    f.log[0] = 255;
    f.inv[0] = 0;
    for (int a = 1; a < 256; ++a) f.inv[a] = f.exp[(255 - f.log[a]) % 255];
    for (int a = 0; a < 256; ++a)
        for (int b = 0; b < 256; ++b)
            f.mul[a][b] = (a == 0 || b == 0) ? 0 : f.exp[f.log[a] + f.log[b]];
    g_ready.store(true, std::memory_order_release);
}
}  // namespace

void field_init() { std::call_once(g_once, build_field); }
bool field_ready() { return g_ready.load(std::memory_order_acquire); }
const Field& field() {
    field_init();
    return g_field;
}

void invert_vandermonde(uint8_t* m, unsigned k) {
    // Restates the recurrence of zfec/fec.c:341-394 exactly (this function is
    // exported as _invert_vdm, so it must return the reference's bytes for
    // ANY input).  The points are p_i = m[i*k+1].  A coefficient vector c of a
    // degree-k polynomial is grown point by point (leading coefficient
    // implicit), then for each point a synthetic division yields the column
    // b and its scale 1/t.  For p_0 = 0 -- the only case fec_new uses, since
    // Vandermonde row 0 is e_0 -- this is the true inverse; for other point
    // sets the reference's recurrence is not, and neither is this one.
    if (k == 1) return;
    const Field& f = field();
    std::vector<uint8_t> p(k), c(k, 0), b(k);
    for (unsigned i = 0; i < k; ++i) p[i] = m[i * k + 1];
    c[k - 1] = p[0];
    for (unsigned i = 1; i < k; ++i) {
        const uint8_t* mul_pi = f.mul[p[i]];
        for (unsigned j = k - i; j + 1 < k; ++j) c[j] ^= mul_pi[c[j + 1]];
        c[k - 1] ^= p[i];
    }
    for (unsigned row = 0; row < k; ++row) {
        const uint8_t* mul_x = f.mul[p[row]];
        uint8_t t = 1;
        b[k - 1] = 1;
        for (unsigned i = k - 1; i > 0; --i) {
            b[i - 1] = c[i] ^ mul_x[b[i]];
            t = mul_x[t] ^ b[i - 1];
        }
        const uint8_t* mul_s = f.mul[f.inv[t]];
        for (unsigned col = 0; col < k; ++col) m[col * k + row] = mul_s[b[col]];
    }
}

void build_encoding_matrix(unsigned k, unsigned n, uint8_t* enc) {
    const Field& f = field();
    std::vector<uint8_t> v(static_cast<size_t>(n) * k, 0);
    v[0] = 1;  // row 0 = e_0 (the first row cannot come from exp[]).
    for (unsigned r = 1; r < n; ++r)
        for (unsigned c = 0; c < k; ++c) v[static_cast<size_t>(r) * k + c] = f.exp[((r - 1) * c) % 255];
    invert_vandermonde(v.data(), k);  // top k x k block -> its inverse
    std::memset(enc, 0, static_cast<size_t>(n) * k);
    for (unsigned c = 0; c < k; ++c) enc[static_cast<size_t>(c) * k + c] = 1;
    for (unsigned r = k; r < n; ++r) {
        const uint8_t* vr = &v[static_cast<size_t>(r) * k];
        uint8_t* er = enc + static_cast<size_t>(r) * k;
        for (unsigned i = 0; i < k; ++i) {
            const uint8_t a = vr[i];
            if (!a) continue;
            const uint8_t* inv_row = &v[static_cast<size_t>(i) * k];
            for (unsigned c = 0; c < k; ++c) er[c] ^= f.mul[a][inv_row[c]];
        }
    }
}

bool invert_matrix(uint8_t* a, unsigned k) {
    // Gauss-Jordan with an augmented identity; the inverse is unique, so any
    // pivot order yields the reference's bytes.
    const Field& f = field();
    const size_t w = 2 * static_cast<size_t>(k);
    thread_local std::vector<uint8_t> aug;  // reused: no allocation per decode call
    aug.assign(static_cast<size_t>(k) * w, 0);
    for (unsigned r = 0; r < k; ++r) {
        std::memcpy(&aug[r * w], a + static_cast<size_t>(r) * k, k);
        aug[r * w + k + r] = 1;
    }
    for (unsigned col = 0; col < k; ++col) {
        unsigned piv = col;
        while (piv < k && aug[piv * w + col] == 0) ++piv;
        if (piv == k) return false;
        if (piv != col)
            for (size_t c = 0; c < w; ++c) std::swap(aug[piv * w + c], aug[col * w + c]);
        uint8_t* prow = &aug[col * w];
        const uint8_t s = f.inv[prow[col]];
        if (s != 1)
            for (size_t c = 0; c < w; ++c) prow[c] = f.mul[s][prow[c]];
        for (unsigned r = 0; r < k; ++r) {
            if (r == col) continue;
            uint8_t* row = &aug[r * w];
            const uint8_t e = row[col];
            if (!e) continue;
            const uint8_t* mrow = f.mul[e];
            for (size_t c = 0; c < w; ++c) row[c] ^= mrow[prow[c]];
        }
    }
    for (unsigned r = 0; r < k; ++r) std::memcpy(a + static_cast<size_t>(r) * k, &aug[r * w + k], k);
    return true;
}

bool build_decode_matrix(const uint8_t* enc, unsigned k, const unsigned* index, uint8_t* dec) {
    for (unsigned i = 0; i < k; ++i) {
        uint8_t* row = dec + static_cast<size_t>(i) * k;
        if (index[i] < k) {
            std::memset(row, 0, k);
            row[i] = 1;
        } else {
            std::memcpy(row, enc + static_cast<size_t>(index[i]) * k, k);
        }
    }
    return invert_matrix(dec, k);
}

}  // namespace zfec_hip
