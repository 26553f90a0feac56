// CPU model of the LZ77 parse's candidate walk (k_lz_local), for design work only: counts the
// candidate batches the speculative chains need on a text block under several index forms.
//   gcc -O2 -o /tmp/lz_sim tools/lz_sim.c && /tmp/lz_sim FILE [MiB]
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef uint32_t u32;
typedef uint8_t u8;
enum { W = 4096, HOME = 4096, CH = 256, LEAD = 48 };
static u32 LPC = 16;

static const u8* T;
static int HB = 10;
static u32 N;

static u32 lcp(u32 p, u32 q, u32 end) {
    u32 l = 0;
    while (p + l < end && T[p + l] == T[q + l]) ++l;
    return l;
}
static u32 h3(u32 x, int hb) {
    u32 k = ((u32)T[x] << 16) | ((u32)T[x + 1] << 8) | T[x + 2];
    return (k * 0x9E3779B1u) >> (32 - hb);
}
static uint64_t key(u32 x, int k) {  // first k bytes big-endian (k <= 8)
    uint64_t v = 0;
    for (int i = 0; i < k; ++i) v = (v << 8) | T[x + i];
    return v;
}

int main(int argc, char** argv) {
    FILE* f = fopen(argv[1], "rb");
    u32 mib = argc > 2 ? atoi(argv[2]) : 1;
    if (argc > 3) HB = atoi(argv[3]);
    if (argc > 4) LPC = atoi(argv[4]);
    N = mib << 20;
    u8* buf = malloc(N + 64);
    N = fread(buf, 1, N, f);
    memset(buf + N, 0, 64);
    T = buf;
    const u32 bs = 1 << 20;
    // stats
    double tok = 0, tok_lead = 0, cand_h10 = 0, cand_ex3 = 0, b_h10 = 0, b_ex3 = 0, wave_b = 0, wave_steps = 0;
    double cand_k[9] = {0}, hist_len[10] = {0}, b_hier = 0, wave_hier = 0, cand_ge[9] = {0};
    for (u32 base = 0; base < N; base += bs) {
        u32 end = base + bs < N ? base + bs : N;
        for (u32 hs = base; hs < end; hs += HOME) {
            u32 nchain = HOME / CH;
            // per chain: list of per-token batch counts
            static u32 bt[16][512], bth[16][512], nt[16];
            for (u32 c = 0; c < nchain; ++c) {
                u32 s = hs + c * CH, e = s + CH < end ? s + CH : end;
                u32 q = (c == 0 && hs == base) ? s : s - LEAD;
                nt[c] = 0;
                while (q < e) {
                    // candidates: window positions x in [max(base, q-W), q) with same hash / 3-gram
                    u32 lo = q - base > W ? q - W : base;
                    u32 best = 0, bd = 0;
                    u32 nh = 0, ne = 0;
                    u32 nk[9] = {0};
                    if (q + 3 <= end) {
                        u32 hq = h3(q, HB);
                        for (u32 x = q; x-- > lo;) {
                            if (h3(x, HB) != hq) continue;
                            ++nh;
                            if (T[x] != T[q] || T[x + 1] != T[q + 1] || T[x + 2] != T[q + 2]) continue;
                            ++ne;
                            u32 l = lcp(q, x, end);
                            for (int k = 3; k <= 8; ++k) if (l >= (u32)k) nk[k]++;
                            if (l > best) best = l, bd = q - x;
                        }
                        // note: the kernel's bucket also holds hash-colliding positions of the
                        // lead region before lo (they stop the walk) -- ignored here
                    }
                    u32 b10 = nh / LPC + 1, b3 = ne / LPC + 1;
                    // hierarchical: 8-gram bucket first (exact keys); if it has an entry the answer
                    // is among them; else 3-gram exact walk but stop at the first candidate when
                    // best can only be 3..7 ... (modelled: walk of the 3-gram bucket entries)
                    u32 bh = nk[8] ? nk[8] / LPC + 1 : 1 + ne / LPC;
                    bt[c][nt[c]] = b10;
                    bth[c][nt[c]] = bh;
                    ++nt[c];
                    tok_lead += 1;
                    if (q >= s) {
                        tok += 1;
                        cand_h10 += nh, cand_ex3 += ne;
                        b_h10 += b10, b_ex3 += b3, b_hier += bh;
                        for (int k = 3; k <= 8; ++k) cand_k[k] += nk[k];
                        hist_len[best >= 3 ? (best < 9 ? best : 9) : 0] += 1;
                    }
                    q += best >= 3 ? best : 1;
                }
            }
            // waves of 4 chains step tokens in lockstep
            for (u32 w = 0; w < nchain / 4; ++w) {
                u32 mx = 0;
                for (u32 g = 0; g < 4; ++g) if (nt[4 * w + g] > mx) mx = nt[4 * w + g];
                for (u32 i = 0; i < mx; ++i) {
                    u32 m = 0, mh = 0;
                    for (u32 g = 0; g < 4; ++g) {
                        u32 c = 4 * w + g;
                        if (i < nt[c]) {
                            if (bt[c][i] > m) m = bt[c][i];
                            if (bth[c][i] > mh) mh = bth[c][i];
                        }
                    }
                    wave_b += m, wave_hier += mh;
                    wave_steps += 1;
                }
            }
        }
    }
    double nw = (double)N / HOME * 4;  // waves
    printf("tokens %.0f (%.2f B/token), with lead-ins %.0f (+%.1f %%)\n", tok, N / tok, tok_lead,
           (tok_lead / tok - 1) * 100);
    printf("per token: hash-10 bucket candidates in window %.2f, exact 3-gram %.2f; >=k:", cand_h10 / tok,
           cand_ex3 / tok);
    for (int k = 3; k <= 8; ++k) printf(" %d:%.2f", k, cand_k[k] / tok);
    printf("\nbatches/token: h10 %.2f ex3 %.2f hier8 %.2f\n", b_h10 / tok, b_ex3 / tok, b_hier / tok);
    printf("per wave: token steps %.1f, batches (lockstep max of 4 chains) h10 %.1f hier8 %.1f\n",
           wave_steps / nw, wave_b / nw, wave_hier / nw);
    printf("match length histogram (0 = literal, 9 = >=9):");
    for (int i = 0; i < 10; ++i) printf(" %d:%.3f", i, hist_len[i] / tok);
    printf("\n");
    return 0;
}
