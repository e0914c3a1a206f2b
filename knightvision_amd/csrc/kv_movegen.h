// Device rules engine: the reference's move generator with every quirk
// (core/chessEngine.py), reformulated on bitboards.
//
// squareUnderAttack(sq) (:400-415) is "sq is the end square of some opponent
// pseudo-move"; here that set is computed whole, as a 64-bit target mask
// (targets()), with occluded fills for the sliders -- so a king-safety probe
// costs one mask instead of a full opponent move list. The legal list is then
// emitted in the reference's exact order (squares r=0..7, c=0..7; per piece the
// reference direction order; king steps then castles) because the sampler
// indexes it (random.choices, self_play.py:162-167).
//
// Every piece of state lives in named scalars (no runtime-indexed arrays), so
// a thread's position stays in registers instead of scratch memory.
//
// Square index s = r*8 + c, row 0 = rank 8. Piece codes: 0 empty, 1..6 wK wQ
// wR wB wN wp, 7..12 bK bQ bR bB bN bp. Types t: 0 K 1 Q 2 R 3 B 4 N 5 P.
#pragma once
#include <stdint.h>

namespace kv {

constexpr int MAXM = 320;  // move-list capacity per position
static_assert(MAXM == KV_MAXM, "include/kv.h KV_MAXM");
constexpr uint64_t FILE_A = 0x0101010101010101ull;
constexpr uint64_t FILE_H = 0x8080808080808080ull;
constexpr uint64_t ROW_1 = 0x000000000000FF00ull;  // row 1 (black pawn start)
constexpr uint64_t ROW_6 = 0x00FF000000000000ull;  // row 6 (white pawn start)

// move word: from | to << 6 | flags << 12; flags bit0 ep, bit1 castle,
// bit2 promotion, bit3 piece moved is a king (Move.pieceMoved[1] == 'K')
constexpr int MF_EP = 1, MF_CASTLE = 2, MF_PROMO = 4, MF_KING = 8;

// flag bits of the state
constexpr int F_WKM = 1, F_BKM = 2, F_WRK = 4, F_WRQ = 8, F_BRK = 16, F_BRQ = 32;

struct Pos {
    uint64_t w, b;                 // occupancy by colour
    uint64_t K, Q, R, B, N, P;     // occupancy by type
    int wtm;
    int wkr, wkc, bkr, bkc;        // stored king locations (stale after a king capture)
    int flags;
    int ep;                        // en-passant square or -1

    __host__ __device__ uint64_t occ(int S) const { return S ? b : w; }
    __host__ __device__ int kr(int S) const { return S ? bkr : wkr; }
    __host__ __device__ int kc(int S) const { return S ? bkc : wkc; }
};

__host__ __device__ inline void pos_set(Pos& p, int sq, int code) {
    const uint64_t m = ~(1ull << sq);
    p.w &= m; p.b &= m;
    p.K &= m; p.Q &= m; p.R &= m; p.B &= m; p.N &= m; p.P &= m;
    if (code > 0) {
        const uint64_t bit = 1ull << sq;
        if (code > 6) p.b |= bit;
        else p.w |= bit;
        switch ((code - 1) % 6) {
            case 0: p.K |= bit; break;
            case 1: p.Q |= bit; break;
            case 2: p.R |= bit; break;
            case 3: p.B |= bit; break;
            case 4: p.N |= bit; break;
            default: p.P |= bit; break;
        }
    }
}

__host__ __device__ inline int pos_at(const Pos& p, int sq) {
    const uint64_t bit = 1ull << sq;
    const int base = (p.w & bit) ? 1 : ((p.b & bit) ? 7 : 0);
    if (!base) return 0;
    const int t = (p.K & bit) ? 0 : (p.Q & bit) ? 1 : (p.R & bit) ? 2 : (p.B & bit) ? 3 : (p.N & bit) ? 4 : 5;
    return base + t;
}

__host__ __device__ inline void pos_from_board(Pos& p, const int8_t* board, int wtm, int wkr, int wkc, int bkr,
                                               int bkc, int flags, int ep) {
    p.w = p.b = p.K = p.Q = p.R = p.B = p.N = p.P = 0;
    for (int s = 0; s < 64; ++s) {
        const int code = board[s];
        if (code > 0) pos_set(p, s, code);
    }
    p.wtm = wtm;
    p.wkr = wkr; p.wkc = wkc; p.bkr = bkr; p.bkc = bkc;
    p.flags = flags;
    p.ep = ep;
}

__host__ __device__ inline void pos_to_board(const Pos& p, int8_t* board) {
    for (int s = 0; s < 64; ++s) board[s] = (int8_t)pos_at(p, s);
}

// ---------------------------------------------------------- fills ----
// D: 0 N(-8) 1 S(+8) 2 W(-1) 3 E(+1) 4 NW(-9) 5 NE(-7) 6 SW(+7) 7 SE(+9);
// east/west steps mask the wrapped file.
template <int D>
__host__ __device__ inline uint64_t shift_dir(uint64_t b) {
    if (D == 0) return b >> 8;
    if (D == 1) return b << 8;
    if (D == 2) return (b >> 1) & ~FILE_H;
    if (D == 3) return (b << 1) & ~FILE_A;
    if (D == 4) return (b >> 9) & ~FILE_H;
    if (D == 5) return (b >> 7) & ~FILE_A;
    if (D == 6) return (b << 7) & ~FILE_H;
    return (b << 9) & ~FILE_A;
}

// squares reached by sliding from `sliders` through `empty`, first blocker included
template <int D>
__host__ __device__ inline uint64_t ray_attacks(uint64_t sliders, uint64_t empty) {
    uint64_t gen = sliders, acc = 0;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        gen = shift_dir<D>(gen);
        acc |= gen;
        gen &= empty;
    }
    return acc;
}

__host__ __device__ inline uint64_t knight_set(uint64_t b) {
    const uint64_t nA = ~FILE_A, nH = ~FILE_H;
    const uint64_t nAB = ~(FILE_A | (FILE_A << 1)), nGH = ~(FILE_H | (FILE_H >> 1));
    return ((b >> 17) & nH) | ((b >> 15) & nA) | ((b >> 10) & nGH) | ((b >> 6) & nAB) | ((b << 17) & nA) |
           ((b << 15) & nH) | ((b << 10) & nAB) | ((b << 6) & nGH);
}

__host__ __device__ inline uint64_t king_set(uint64_t b) {
    uint64_t a = (b >> 8) | (b << 8);
    const uint64_t w = (b >> 1) & ~FILE_H, e = (b << 1) & ~FILE_A;
    a |= w | e | (w >> 8) | (w << 8) | (e >> 8) | (e << 8);
    return a;
}

__host__ __device__ inline int ctz64(uint64_t x) {
#ifdef __HIP_DEVICE_COMPILE__
    return __ffsll((unsigned long long)x) - 1;
#else
    return __builtin_ctzll(x);
#endif
}

// End squares of every pseudo-move of side S (0 white, 1 black) on this
// board: squareUnderAttack's opponent move list (:405-415), including pawn
// pushes, pawn "captures" onto the en-passant square, unfiltered king steps
// and castle destinations (nested probes return False, :401-403). Knight and
// king sets are the union over all such pieces (one fill each).
__host__ __device__ inline uint64_t targets(const Pos& p, int S) {
    const uint64_t own = p.occ(S), opp = p.occ(S ^ 1);
    const uint64_t empty = ~(own | opp);
    const uint64_t epb = p.ep >= 0 ? (1ull << p.ep) : 0ull;
    uint64_t t = 0;
    const uint64_t Pw = p.P & own;
    if (S == 0) {
        t |= ((Pw >> 8) & empty) | ((((Pw & ROW_6) >> 8) & empty) >> 8 & empty);
        t |= (((Pw & ~FILE_A) >> 9) | ((Pw & ~FILE_H) >> 7)) & (opp | epb);
    } else {
        t |= ((Pw << 8) & empty) | ((((Pw & ROW_1) << 8) & empty) << 8 & empty);
        t |= (((Pw & ~FILE_A) << 7) | ((Pw & ~FILE_H) << 9)) & (opp | epb);
    }
    const uint64_t Ks = p.K & own;
    t |= (knight_set(p.N & own) | king_set(Ks)) & ~own;
    const uint64_t rq = (p.R | p.Q) & own, bq = (p.B | p.Q) & own;
    const uint64_t sl = ray_attacks<0>(rq, empty) | ray_attacks<1>(rq, empty) | ray_attacks<2>(rq, empty) |
                        ray_attacks<3>(rq, empty) | ray_attacks<4>(bq, empty) | ray_attacks<5>(bq, empty) |
                        ray_attacks<6>(bq, empty) | ray_attacks<7>(bq, empty);
    t |= sl & ~own;
    if (Ks) {  // getCastleMoves (:575-601) for side S; every inner probe is False
        const int row = S == 0 ? 7 : 0;
        const int kmoved = S == 0 ? (p.flags & F_WKM) : (p.flags & F_BKM);
        if (p.kr(S) == row && p.kc(S) == 4 && !kmoved) {
            const int rk = S == 0 ? (p.flags & F_WRK) : (p.flags & F_BRK);
            const int rqf = S == 0 ? (p.flags & F_WRQ) : (p.flags & F_BRQ);
            const int base = row * 8;
            const uint64_t rook = p.R & own;
            if (!rk && (empty >> (base + 5) & 1) && (empty >> (base + 6) & 1) && (rook >> (base + 7) & 1))
                t |= 1ull << (base + 6);
            if (!rqf && (empty >> (base + 1) & 1) && (empty >> (base + 2) & 1) && (empty >> (base + 3) & 1) &&
                (rook >> (base + 0) & 1))
                t |= 1ull << (base + 2);
        }
    }
    return t;
}

// ------------------------------------------- wave-cooperative generator ----
// One wavefront per position, lane = square (the reference's enumeration
// order r=0..7, c=0..7 is lane order). Every lane holds the same Pos (built
// from ballots); each lane generates the moves of the piece on its square as
// a destination mask, the legality filters are mask operations, an exclusive
// wave scan of the per-lane counts gives each lane its slot in the ordered
// list, and the lane writes its moves in the reference's per-piece order.

__constant__ const int8_t kKnightD[8][2] = {{-2, -1}, {-1, -2}, {-2, 1}, {-1, 2}, {1, -2}, {2, -1}, {1, 2}, {2, 1}};
__constant__ const int8_t kKingD[8][2] = {{-1, -1}, {-1, 0}, {-1, 1}, {0, -1}, {0, 1}, {1, -1}, {1, 0}, {1, 1}};
// rook rays :478 then bishop rays :517 (queen = both, :536-538); also the
// ray order of checkForPinsAndChecks :331
__constant__ const int8_t kSlideD[8][2] = {{-1, 0}, {1, 0}, {0, -1}, {0, 1}, {-1, -1}, {-1, 1}, {1, -1}, {1, 1}};
__constant__ const int8_t kPinD[8][2] = {{-1, 0}, {0, -1}, {1, 0}, {0, 1}, {-1, -1}, {-1, 1}, {1, -1}, {1, 1}};
__constant__ const int8_t kKChkD[7][2] = {{-2, -1}, {-1, -2}, {-1, 2}, {1, -2}, {2, -1}, {1, 2}, {2, 1}};  // Q1

__device__ inline bool inb(int r, int c) { return (unsigned)r < 8u && (unsigned)c < 8u; }

__device__ inline Pos wave_pos(int code, int wtm, int wkr, int wkc, int bkr, int bkc, int flags, int ep) {
    Pos p;
    const int t = code > 0 ? (code - 1) % 6 : -1;
    p.w = __ballot(code >= 1 && code <= 6);
    p.b = __ballot(code >= 7);
    p.K = __ballot(t == 0);
    p.Q = __ballot(t == 1);
    p.R = __ballot(t == 2);
    p.B = __ballot(t == 3);
    p.N = __ballot(t == 4);
    p.P = __ballot(t == 5);
    p.wtm = wtm;
    p.wkr = wkr; p.wkc = wkc; p.bkr = bkr; p.bkc = bkc;
    p.flags = flags;
    p.ep = ep;
    return p;
}

__device__ inline uint64_t wave_or(uint64_t v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v |= __shfl_xor(v, m);
    return v;
}

__device__ inline int wave_excl_scan(int v, int lane, int& total) {
    int x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    total = __shfl(x, 63);
    return x - v;
}

// Move.__init__ flags (:693-713): promotion by the moved pawn's colour, king
// moves flagged for the in-check filter
__device__ inline uint16_t move_word(const Pos& p, int fr, int to, int fl) {
    const uint64_t fb = 1ull << fr;
    if ((p.P & fb) && (((p.w & fb) && to < 8) || ((p.b & fb) && to >= 56))) fl |= MF_PROMO;
    if (p.K & fb) fl |= MF_KING;
    return (uint16_t)(fr | (to << 6) | (fl << 12));
}

// squares (r',c') with (r'-r)*pdc == (c'-c)*pdr: the pin line through (r,c)
__device__ inline uint64_t pin_line(int r, int c, int pdr, int pdc) {
    if (pdr == 0) return 0xFFull << (8 * r);
    if (pdc == 0) return FILE_A << c;
    if (pdr == pdc) {
        const int d = r - c;
        return d >= 0 ? 0x8040201008040201ull << (8 * d) : 0x8040201008040201ull >> (-8 * d);
    }
    const int t = r + c;
    return t >= 7 ? 0x0102040810204080ull << (8 * (t - 7)) : 0x0102040810204080ull >> (8 * (7 - t));
}

// getKingMoves :543-573 king-step probes for the king on `src`, one probe per
// lane 0..7: the probe moves the king, asks whether the opponent reaches the
// destination, and restores board[src] = the king -- literally, so a stale
// king location (src without a king) gets a king written to it, as the
// reference does. Returns the 8-bit mask of passing probes (all lanes).
__device__ inline uint32_t wave_king_probes(Pos& p, int src, int lane) {
    const int S = p.wtm ? 0 : 1;
    const int kcode = S == 0 ? 1 : 7;
    bool ok = false, ran = false;
    if (lane < 8) {
        const int er = (src >> 3) + kKingD[lane][0], ec = (src & 7) + kKingD[lane][1];
        if (inb(er, ec)) {
            const int dst = er * 8 + ec;
            if (!((p.occ(S) >> dst) & 1)) {
                ran = true;
                Pos q = p;
                pos_set(q, src, 0);
                pos_set(q, dst, kcode);
                ok = !((targets(q, S ^ 1) >> dst) & 1);
            }
        }
    }
    const uint64_t okm = __ballot(ok);
    if (__ballot(ran)) pos_set(p, src, kcode);
    return (uint32_t)(okm & 0xFF);
}

// getCastleMoves :575-601 for a king probed on `src` (att = opponent targets
// on the board after the probes). Bit 0 king side, bit 1 queen side.
__device__ inline uint32_t castle_bits(const Pos& p, int src, uint64_t att) {
    const int S = p.wtm ? 0 : 1;
    if ((att >> src) & 1) return 0;
    const int row = S == 0 ? 7 : 0;
    const int kmoved = S == 0 ? (p.flags & F_WKM) : (p.flags & F_BKM);
    if (!(p.kr(S) == row && p.kc(S) == 4) || kmoved) return 0;
    const uint64_t all = p.w | p.b;
    const int base = row * 8;
    const uint64_t rook = p.R & p.occ(S);
    const int rk = S == 0 ? (p.flags & F_WRK) : (p.flags & F_BRK);
    const int rq = S == 0 ? (p.flags & F_WRQ) : (p.flags & F_BRQ);
    uint32_t cb = 0;
    if (!rk && !((all >> (base + 5)) & 1) && !((all >> (base + 6)) & 1) && !((att >> (base + 5)) & 1) &&
        !((att >> (base + 6)) & 1) && ((rook >> (base + 7)) & 1))
        cb |= 1;
    if (!rq && !((all >> (base + 1)) & 1) && !((all >> (base + 2)) & 1) && !((all >> (base + 3)) & 1) &&
        !((att >> (base + 2)) & 1) && !((att >> (base + 3)) & 1) && ((rook >> (base + 0)) & 1))
        cb |= 2;
    return cb;
}

// getValidMoves :277-321 for the position every lane holds. Writes the ordered
// list to out[0 .. min(n, cap)), returns n (all lanes; n > cap = overflow).
// May mutate p (the stale-king write of the double-check branch); callers
// store the board back.
__device__ inline int wave_valid_moves(Pos& p, uint16_t* out, int cap, int lane) {
    const int S = p.wtm ? 0 : 1, E = S ^ 1;
    const int kr = p.kr(S), kc = p.kc(S);
    const uint64_t own = p.occ(S), opp = p.occ(E);
    const int base = S == 0 ? 56 : 0;

    // checkForPinsAndChecks :325-383: lanes 0..7 one ray each, 8..14 the
    // seven knight offsets (Q1)
    int pinned_sq = -1, hit = 0, hr = 0, hc = 0, hdr = 0, hdc = 0;
    if (lane < 8) {
        const int dr = kPinD[lane][0], dc = kPinD[lane][1];
        const bool orth = lane < 4;
        int cand = -1;
        for (int i = 1; i < 8; ++i) {
            const int er = kr + dr * i, ec = kc + dc * i;
            if (!inb(er, ec)) break;
            const int sq = er * 8 + ec;
            const uint64_t bit = 1ull << sq;
            if (own & bit) {
                if (cand < 0) cand = sq;
                else break;
            } else if (opp & bit) {
                const bool rq = ((p.R | p.Q) & bit) != 0, bq = ((p.B | p.Q) & bit) != 0, pawn = (p.P & bit) != 0;
                const bool h = (orth && rq) || (!orth && bq) ||
                               (i == 1 && pawn && !orth && ((E == 0 && dr == 1) || (E == 1 && dr == -1)));
                if (h) {
                    if (cand < 0) {
                        hit = 1; hr = er; hc = ec; hdr = dr; hdc = dc;
                    } else {
                        pinned_sq = cand;
                    }
                }
                break;
            }
        }
    } else if (lane < 15) {
        const int er = kr + kKChkD[lane - 8][0], ec = kc + kKChkD[lane - 8][1];
        if (inb(er, ec) && (((opp & p.N) >> (er * 8 + ec)) & 1)) {
            hit = 1; hr = er; hc = ec; hdr = kKChkD[lane - 8][0]; hdc = kKChkD[lane - 8][1];
        }
    }
    const uint64_t hits = __ballot(hit);
    const int nchk = __popcll(hits);

    if (nchk >= 2) {  // double check: getKingMoves on the stored king square only (:312-313)
        const int src = kr * 8 + kc;
        const uint32_t kb = wave_king_probes(p, src, lane);
        const uint32_t cb = castle_bits(p, src, targets(p, E));
        bool has = false;
        int fr = src, to = 0, fl = 0;
        if (lane < 8) {
            has = (kb >> lane) & 1;
            to = src + kKingD[lane][0] * 8 + kKingD[lane][1];
        } else if (lane == 8) {
            has = cb & 1; fr = base + 4; to = base + 6; fl = MF_CASTLE;
        } else if (lane == 9) {
            has = (cb >> 1) & 1; fr = base + 4; to = base + 2; fl = MF_CASTLE;
        }
        const uint64_t hm = __ballot(has);
        if (has) {
            const int off = __popcll(hm & ((1ull << lane) - 1));
            if (off < cap) out[off] = move_word(p, fr, to, fl);
        }
        return __popcll(hm);
    }

    const uint64_t pinned = wave_or(pinned_sq >= 0 ? 1ull << pinned_sq : 0ull);
    const uint64_t att = targets(p, E);  // the board is unchanged below: probes run on real kings

    // king probes for each of the mover's kings (normally one)
    uint32_t my_kb = 0;
    for (uint64_t ks = p.K & own; ks; ks &= ks - 1) {
        const int s = ctz64(ks);
        const uint32_t kb = wave_king_probes(p, s, lane) | (castle_bits(p, s, att) << 8);
        if (lane == s) my_kb = kb;
    }

    // this lane's piece: destination mask M (+ castle bits cb)
    const uint64_t me = 1ull << lane;
    const int r = lane >> 3, c = lane & 7;
    const uint64_t empty = ~(p.w | p.b);
    int t = -1;
    if (own & me) t = (p.K & me) ? 0 : (p.Q & me) ? 1 : (p.R & me) ? 2 : (p.B & me) ? 3 : (p.N & me) ? 4 : 5;
    const bool pin = (pinned & me) != 0;
    const int pdr = pin ? (r > kr) - (r < kr) : 0, pdc = pin ? (c > kc) - (c < kc) : 0;
    const int ma = p.wtm ? -1 : 1;
    uint64_t M = 0;
    uint32_t cb = 0;
    if (t == 5) {  // getPawnMoves :447-472
        const int start = p.wtm ? 6 : 1;
        if ((unsigned)(r + ma) < 8u) {
            if (!pin || (pdr == ma && pdc == 0)) {
                const int to1 = (r + ma) * 8 + c;
                if ((empty >> to1) & 1) {
                    M |= 1ull << to1;
                    if (r == start && ((empty >> (to1 + ma * 8)) & 1)) M |= 1ull << (to1 + ma * 8);
                }
            }
            if (c > 0 && (!pin || (pdr == ma && pdc == -1))) {
                const int to = (r + ma) * 8 + c - 1;
                if (((opp >> to) & 1) || to == p.ep) M |= 1ull << to;
            }
            if (c < 7 && (!pin || (pdr == ma && pdc == 1))) {
                const int to = (r + ma) * 8 + c + 1;
                if (((opp >> to) & 1) || to == p.ep) M |= 1ull << to;
            }
        }
    } else if (t == 4) {  // getKnightMoves :500-512; a pinned knight has none (:618)
        if (!pin) M = knight_set(me) & ~own;
    } else if (t >= 1) {  // rook / bishop / queen rays
        uint64_t a = 0;
        if (t != 3)
            a |= ray_attacks<0>(me, empty) | ray_attacks<1>(me, empty) | ray_attacks<2>(me, empty) |
                 ray_attacks<3>(me, empty);
        if (t != 2)
            a |= ray_attacks<4>(me, empty) | ray_attacks<5>(me, empty) | ray_attacks<6>(me, empty) |
                 ray_attacks<7>(me, empty);
        M = a & ~own;
    } else if (t == 0) {
        for (int k = 0; k < 8; ++k)
            if ((my_kb >> k) & 1) M |= 1ull << (lane + kKingD[k][0] * 8 + kKingD[k][1]);
        cb = (my_kb >> 8) & 3;
    }
    if (pin) {  // addPieceMovesConsideringPins :604-630: keep moves along the pin line
        const uint64_t line = pin_line(r, c, pdr, pdc);
        M &= line;
        if (!((line >> (base + 6)) & 1)) cb &= ~1u;
        if (!((line >> (base + 2)) & 1)) cb &= ~2u;
    }
    if (nchk == 1) {  // single check (:291-310): block / capture squares, king moves re-probed
        const int first = ctz64(hits);
        const int cr = __shfl(hr, first), cc = __shfl(hc, first);
        const int cdr = __shfl(hdr, first), cdc = __shfl(hdc, first);
        uint64_t valid = 0;
        if ((p.N >> (cr * 8 + cc)) & 1) {
            valid = 1ull << (cr * 8 + cc);
        } else {
            for (int i = 1; i < 8; ++i) {
                const int sr = kr + cdr * i, sc = kc + cdc * i;
                if (inb(sr, sc)) valid |= 1ull << (sr * 8 + sc);
                if (sr == cr && sc == cc) break;
            }
        }
        M &= t == 0 ? ~att : valid;
        const bool kfrom = (p.K >> (base + 4)) & 1;  // castle moves start on base+4
        const uint64_t keep = kfrom ? ~att : valid;
        if (!((keep >> (base + 6)) & 1)) cb &= ~1u;
        if (!((keep >> (base + 2)) & 1)) cb &= ~2u;
    }

    int total;
    int w = wave_excl_scan(__popcll(M) + __popc(cb), lane, total);
    auto emit = [&](int fr, int to, int fl) {
        if (w < cap) out[w] = move_word(p, fr, to, fl);
        ++w;
    };
    if (t == 5) {  // push1, push2, capture c-1, capture c+1 (en passant when the square is empty)
        if ((unsigned)(r + ma) < 8u) {
            const int to1 = (r + ma) * 8 + c;
            if ((M >> to1) & 1) emit(lane, to1, 0);
            if ((unsigned)(r + 2 * ma) < 8u && ((M >> (to1 + ma * 8)) & 1)) emit(lane, to1 + ma * 8, 0);
            if (c > 0 && ((M >> (to1 - 1)) & 1)) emit(lane, to1 - 1, ((opp >> (to1 - 1)) & 1) ? 0 : MF_EP);
            if (c < 7 && ((M >> (to1 + 1)) & 1)) emit(lane, to1 + 1, ((opp >> (to1 + 1)) & 1) ? 0 : MF_EP);
        }
    } else if (t == 4) {
        for (int k = 0; k < 8; ++k) {
            const int er = r + kKnightD[k][0], ec = c + kKnightD[k][1];
            if (inb(er, ec) && ((M >> (er * 8 + ec)) & 1)) emit(lane, er * 8 + ec, 0);
        }
    } else if (t >= 1) {
        const int k0 = t == 3 ? 4 : 0, k1 = t == 2 ? 4 : 8;
        for (int k = k0; k < k1; ++k) {
            const int dr = kSlideD[k][0], dc = kSlideD[k][1];
            for (int i = 1; i < 8; ++i) {
                const int er = r + dr * i, ec = c + dc * i;
                if (!inb(er, ec)) break;
                if ((M >> (er * 8 + ec)) & 1) emit(lane, er * 8 + ec, 0);
            }
        }
    } else if (t == 0) {
        for (int k = 0; k < 8; ++k) {
            const int er = r + kKingD[k][0], ec = c + kKingD[k][1];
            if (inb(er, ec) && ((M >> (er * 8 + ec)) & 1)) emit(lane, er * 8 + ec, 0);
        }
        if (cb & 1) emit(base + 4, base + 6, MF_CASTLE);
        if (cb & 2) emit(base + 4, base + 2, MF_CASTLE);
    }
    return total;
}


// inCheck :388-394
__device__ inline bool in_check(const Pos& p) {
    const int S = p.wtm ? 0 : 1;
    const int kr = p.kr(S), kc = p.kc(S);
    if (!inb(kr, kc)) return false;
    return (targets(p, S ^ 1) >> (kr * 8 + kc)) & 1;
}

// makeMove :127-197 on a mailbox board + the bookkeeping fields.
__host__ __device__ inline void make_move_board(int8_t* b, int& wtm, int& wkr, int& wkc, int& bkr, int& bkc,
                                                int& flags, int& ep, int mv) {
    const int fr = mv & 63, to = (mv >> 6) & 63, fl = (mv >> 12) & 15;
    const int moved = b[fr];
    b[fr] = 0;
    b[to] = (int8_t)moved;
    if (moved == 1) flags |= F_WKM;
    else if (moved == 7) flags |= F_BKM;
    else if (moved == 3) {
        if (fr == 56) flags |= F_WRQ;
        else if (fr == 63) flags |= F_WRK;
    } else if (moved == 9) {
        if (fr == 0) flags |= F_BRQ;
        else if (fr == 7) flags |= F_BRK;
    }
    if (fl & MF_EP) b[(fr & ~7) | (to & 7)] = 0;
    if (fl & MF_CASTLE) {
        const int row = to & ~7, tc = to & 7, fc = fr & 7;
        if (tc - fc == 2) {
            b[row + tc - 1] = b[row + tc + 1];
            b[row + tc + 1] = 0;
        } else {
            b[row + tc + 1] = b[row + tc - 2];
            b[row + tc - 2] = 0;
        }
    }
    const int fr_r = fr >> 3, to_r = to >> 3;
    if (moved > 0 && (moved - 1) % 6 == 5 && (fr_r - to_r == 2 || to_r - fr_r == 2))
        ep = ((fr_r + to_r) / 2) * 8 + (fr & 7);
    else
        ep = -1;
    wtm = !wtm;
    if (moved == 1) { wkr = to_r; wkc = to & 7; }
    else if (moved == 7) { bkr = to_r; bkc = to & 7; }
    if (fl & MF_PROMO) b[to] = (int8_t)(moved <= 6 ? 2 : 8);
}

// GameState.isDraw :21-33: only kings (or nothing) left
__host__ __device__ inline bool is_draw_board(const int8_t* b) {
    for (int s = 0; s < 64; ++s)
        if (b[s] != 0 && b[s] != 1 && b[s] != 7) return false;
    return true;
}

}  // namespace kv
