// gf256.cpp -- host GF(2^8) tables (restated from gf256.cpp:366-460 of the reference; the
// construction is the textbook exp/log one for polynomial 0x14D).
#include "gf256.h"

#include <string.h>

namespace tamd {

GF g_gf;

static bool self_test() {
    // Same consistency checks the reference runs at init (gf256.cpp:84-121).
    for (unsigned i = 0; i < 256; ++i) {
        for (unsigned j = 0; j < 256; ++j) {
            const uint8_t p = gf_mul((uint8_t)i, (uint8_t)j);
            if (i && j) {
                if (gf_div(p, (uint8_t)i) != j || gf_div(p, (uint8_t)j) != i) return false;
            } else if (p != 0) {
                return false;
            }
            if (j == 1 && p != i) return false;
        }
    }
    // Known answers.
    return gf_mul(2, 0x80) == 0x4d && gf_mul(0xaa, 0x6c) == 0x7c && gf_inv(2) == 0xa6 && gf_sqr(3) == 5;
}

bool gf_init() {
    if (g_gf.ready) return true;
    const unsigned poly = 0x14d;
    uint8_t exp[1024];
    uint16_t log[256];
    memset(exp, 0, sizeof(exp));
    log[0] = 512;
    unsigned v = 1;
    for (unsigned j = 0; j < 255; ++j) {
        exp[j] = (uint8_t)v;
        log[v] = (uint16_t)j;
        v <<= 1;
        if (v & 0x100) v ^= poly;
    }
    for (unsigned j = 255; j < 510; ++j) exp[j] = exp[j - 255];
    exp[510] = 1;

    for (unsigned x = 0; x < 256; ++x) {
        g_gf.mul[0][x] = 0;
        g_gf.div[0][x] = 0;
    }
    for (unsigned y = 1; y < 256; ++y) {
        const unsigned ly = log[y];
        for (unsigned x = 0; x < 256; ++x) {
            if (x == 0) { g_gf.mul[y][0] = 0; g_gf.div[y][0] = 0; continue; }
            g_gf.mul[y][x] = exp[log[x] + ly];
            g_gf.div[y][x] = exp[log[x] + 255 - ly];
        }
    }
    for (unsigned x = 0; x < 256; ++x) {
        g_gf.inv[x] = g_gf.div[x][1];
        g_gf.sqr[x] = g_gf.mul[x][x];
    }
    for (unsigned c = 0; c < 256; ++c) {
        uint8_t t[3][8];
        for (unsigned i = 0; i < 8; ++i) {
            t[0][i] = g_gf.mul[c][i];
            t[1][i] = g_gf.mul[c][i << 3];
            t[2][i] = i < 4 ? g_gf.mul[c][i << 6] : 0;
        }
        memcpy(&g_gf.perm[c][0], t, 24);
        g_gf.perm[c][6] = 0;
        g_gf.perm[c][7] = 0;
    }
    g_gf.ready = self_test();
    return g_gf.ready;
}

} // namespace tamd
