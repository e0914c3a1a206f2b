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
// Square index s = r*8 + c, row 0 = rank 8. Piece codes: 0 empty, 1..6 wK wQ
// wR wB wN wp, 7..12 bK bQ bR bB bN bp. Types t: 0 K 1 Q 2 R 3 B 4 N 5 P.
#pragma once
#include <stdint.h>

namespace kv {

constexpr int MAXM = 320;  // move-list capacity per position
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
    uint64_t occ[2];  // [0] white, [1] black
    uint64_t pc[6];   // K Q R B N P
    int wtm;
    int kr[2], kc[2];  // stored king locations (stale after a king capture)
    int flags;
    int ep;  // en-passant square or -1
};

// 80-byte state vector <-> Pos (layout: oracle/kv_oracle.c header)
struct StateVec {
    int8_t v[80];
};

__host__ __device__ inline void pos_set(Pos& p, int sq, int code) {
    const uint64_t b = 1ull << sq;
    p.occ[0] &= ~b;
    p.occ[1] &= ~b;
#pragma unroll
    for (int t = 0; t < 6; ++t) p.pc[t] &= ~b;
    if (code > 0) {
        p.occ[code > 6 ? 1 : 0] |= b;
        p.pc[(code - 1) % 6] |= b;
    }
}

__host__ __device__ inline int pos_at(const Pos& p, int sq) {
    const uint64_t b = 1ull << sq;
    const int col = (p.occ[0] & b) ? 0 : ((p.occ[1] & b) ? 1 : -1);
    if (col < 0) return 0;
    int t = 0;
    while (t < 5 && !(p.pc[t] & b)) ++t;
    return col * 6 + t + 1;
}

__host__ __device__ inline void pos_from_board(Pos& p, const int8_t* board, int wtm, int wkr, int wkc, int bkr,
                                               int bkc, int flags, int ep) {
    p.occ[0] = p.occ[1] = 0;
    for (int t = 0; t < 6; ++t) p.pc[t] = 0;
    for (int s = 0; s < 64; ++s) {
        const int code = board[s];
        if (code > 0) {
            p.occ[code > 6 ? 1 : 0] |= 1ull << s;
            p.pc[(code - 1) % 6] |= 1ull << s;
        }
    }
    p.wtm = wtm;
    p.kr[0] = wkr; p.kc[0] = wkc; p.kr[1] = bkr; p.kc[1] = bkc;
    p.flags = flags;
    p.ep = ep;
}

__host__ __device__ inline void pos_to_board(const Pos& p, int8_t* board) {
    for (int s = 0; s < 64; ++s) board[s] = (int8_t)pos_at(p, s);
}

// ---------------------------------------------------------- fills ----
// occluded fill of `gen` through `pro` along one direction, then one more step
// (the first blocker is included); east/west steps mask the wrapped file.
template <int D>
__host__ __device__ inline uint64_t shift_dir(uint64_t b) {
    // D: 0 N(-8) 1 S(+8) 2 W(-1) 3 E(+1) 4 NW(-9) 5 NE(-7) 6 SW(+7) 7 SE(+9)
    if (D == 0) return b >> 8;
    if (D == 1) return b << 8;
    if (D == 2) return (b >> 1) & ~FILE_H;
    if (D == 3) return (b << 1) & ~FILE_A;
    if (D == 4) return (b >> 9) & ~FILE_H;
    if (D == 5) return (b >> 7) & ~FILE_A;
    if (D == 6) return (b << 7) & ~FILE_H;
    return (b << 9) & ~FILE_A;
}

template <int D>
__host__ __device__ inline uint64_t ray_attacks(uint64_t sliders, uint64_t empty) {
    uint64_t gen = sliders, acc = 0;
    // plain iterative fill: 7 steps at most
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        gen = shift_dir<D>(gen);
        acc |= gen;
        gen &= empty;
    }
    return acc;
}

__host__ __device__ inline uint64_t knight_att(int s) {
    const uint64_t b = 1ull << s;
    const uint64_t nA = ~FILE_A, nH = ~FILE_H;
    const uint64_t nAB = ~(FILE_A | (FILE_A << 1)), nGH = ~(FILE_H | (FILE_H >> 1));
    return ((b >> 17) & nH) | ((b >> 15) & nA) | ((b >> 10) & nGH) | ((b >> 6) & nAB) | ((b << 17) & nA) |
           ((b << 15) & nH) | ((b << 10) & nAB) | ((b << 6) & nGH);
}

__host__ __device__ inline uint64_t king_att(int s) {
    const uint64_t b = 1ull << s;
    uint64_t a = (b >> 8) | (b << 8);
    const uint64_t w = (b >> 1) & ~FILE_H, e = (b << 1) & ~FILE_A;
    a |= w | e | (w >> 8) | (w << 8) | (e >> 8) | (e << 8);
    return a;
}

__host__ __device__ inline int popc64(uint64_t x) {
#ifdef __HIP_DEVICE_COMPILE__
    return __popcll(x);
#else
    return __builtin_popcountll(x);
#endif
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
// and castle destinations (nested probes return False, :401-403).
__host__ __device__ inline uint64_t targets(const Pos& p, int S) {
    const uint64_t own = p.occ[S], opp = p.occ[S ^ 1];
    const uint64_t empty = ~(own | opp);
    const uint64_t epb = p.ep >= 0 ? (1ull << p.ep) : 0ull;
    uint64_t t = 0;
    const uint64_t P = p.pc[5] & own;
    if (S == 0) {
        const uint64_t p1 = (P >> 8) & empty;
        t |= p1 | ((((P & ROW_6) >> 8) & empty) >> 8 & empty);
        t |= (((P & ~FILE_A) >> 9) | ((P & ~FILE_H) >> 7)) & (opp | epb);
    } else {
        const uint64_t p1 = (P << 8) & empty;
        t |= p1 | ((((P & ROW_1) << 8) & empty) << 8 & empty);
        t |= (((P & ~FILE_A) << 7) | ((P & ~FILE_H) << 9)) & (opp | epb);
    }
    for (uint64_t n = p.pc[4] & own; n; n &= n - 1) t |= knight_att(ctz64(n)) & ~own;
    const uint64_t K = p.pc[0] & own;
    for (uint64_t k = K; k; k &= k - 1) t |= king_att(ctz64(k)) & ~own;
    const uint64_t rq = (p.pc[2] | p.pc[1]) & own, bq = (p.pc[3] | p.pc[1]) & own;
    uint64_t sl = ray_attacks<0>(rq, empty) | ray_attacks<1>(rq, empty) | ray_attacks<2>(rq, empty) |
                  ray_attacks<3>(rq, empty) | ray_attacks<4>(bq, empty) | ray_attacks<5>(bq, empty) |
                  ray_attacks<6>(bq, empty) | ray_attacks<7>(bq, empty);
    t |= sl & ~own;
    if (K) {  // getCastleMoves (:575-601) for side S; every inner probe is False
        const int row = S == 0 ? 7 : 0;
        const int kmoved = S == 0 ? (p.flags & F_WKM) : (p.flags & F_BKM);
        if (p.kr[S] == row && p.kc[S] == 4 && !kmoved) {
            const int rk = S == 0 ? (p.flags & F_WRK) : (p.flags & F_BRK);
            const int rqf = S == 0 ? (p.flags & F_WRQ) : (p.flags & F_BRQ);
            const int base = row * 8;
            const uint64_t rook = p.pc[2] & own;
            if (!rk && (empty >> (base + 5) & 1) && (empty >> (base + 6) & 1) && (rook >> (base + 7) & 1))
                t |= 1ull << (base + 6);
            if (!rqf && (empty >> (base + 1) & 1) && (empty >> (base + 2) & 1) && (empty >> (base + 3) & 1) &&
                (rook >> (base + 0) & 1))
                t |= 1ull << (base + 2);
        }
    }
    return t;
}

// ------------------------------------------------------ move emission ----
struct MoveOut {
    uint16_t* m;
    int n;
    int cap;
    int overflow;
    __host__ __device__ inline void add(const Pos& p, int fr, int to, int fl) {
        const int moved = pos_at(p, fr);
        if (moved > 0 && (moved - 1) % 6 == 5) {
            if ((moved <= 6 && to < 8) || (moved > 6 && to >= 56)) fl |= MF_PROMO;
        }
        if (moved > 0 && (moved - 1) % 6 == 0) fl |= MF_KING;
        if (n < cap) m[n] = (uint16_t)(fr | (to << 6) | (fl << 12));
        else overflow = 1;
        ++n;
    }
};

__constant__ const int8_t kRookD[4][2] = {{-1, 0}, {1, 0}, {0, -1}, {0, 1}};
__constant__ const int8_t kBishD[4][2] = {{-1, -1}, {-1, 1}, {1, -1}, {1, 1}};
__constant__ const int8_t kKnightD[8][2] = {{-2, -1}, {-1, -2}, {-2, 1}, {-1, 2}, {1, -2}, {2, -1}, {1, 2}, {2, 1}};
__constant__ const int8_t kKingD[8][2] = {{-1, -1}, {-1, 0}, {-1, 1}, {0, -1}, {0, 1}, {1, -1}, {1, 0}, {1, 1}};
__constant__ const int8_t kPinD[8][2] = {{-1, 0}, {0, -1}, {1, 0}, {0, 1}, {-1, -1}, {-1, 1}, {1, -1}, {1, 1}};
__constant__ const int8_t kKChkD[7][2] = {{-2, -1}, {-1, -2}, {-1, 2}, {1, -2}, {2, -1}, {1, 2}, {2, 1}};

__device__ inline bool inb(int r, int c) { return (unsigned)r < 8u && (unsigned)c < 8u; }

// sliding moves in the reference's ray order (getRookMoves :477-494,
// getBishopMoves :516-531)
__device__ inline void slide_moves(const Pos& p, int r, int c, const int8_t (*dirs)[2], MoveOut& o) {
    const int S = p.wtm ? 0 : 1;
    for (int k = 0; k < 4; ++k) {
        for (int i = 1; i < 8; ++i) {
            const int er = r + dirs[k][0] * i, ec = c + dirs[k][1] * i;
            if (!inb(er, ec)) break;
            const uint64_t b = 1ull << (er * 8 + ec);
            if (p.occ[S] & b) break;
            o.add(p, r * 8 + c, er * 8 + ec, 0);
            if (p.occ[S ^ 1] & b) break;
        }
    }
}

// getPawnMoves :447-472 (pin = direction or null)
__device__ inline void pawn_moves(const Pos& p, int r, int c, const int* pin, MoveOut& o) {
    const int S = p.wtm ? 0 : 1;
    const int ma = p.wtm ? -1 : 1, start = p.wtm ? 6 : 1;
    const uint64_t all = p.occ[0] | p.occ[1];
    if (!pin || (pin[0] == ma && pin[1] == 0)) {
        if ((unsigned)(r + ma) < 8u && !((all >> ((r + ma) * 8 + c)) & 1)) {
            o.add(p, r * 8 + c, (r + ma) * 8 + c, 0);
            if (r == start && !((all >> ((r + 2 * ma) * 8 + c)) & 1)) o.add(p, r * 8 + c, (r + 2 * ma) * 8 + c, 0);
        }
    }
    for (int k = 0; k < 2; ++k) {
        const int dc = k ? 1 : -1;
        if ((unsigned)(c + dc) < 8u && (!pin || (pin[0] == ma && pin[1] == dc)) && (unsigned)(r + ma) < 8u) {
            const int to = (r + ma) * 8 + c + dc;
            if ((p.occ[S ^ 1] >> to) & 1) o.add(p, r * 8 + c, to, 0);
            else if (to == p.ep) o.add(p, r * 8 + c, to, MF_EP);
        }
    }
}

__device__ inline void knight_moves(const Pos& p, int r, int c, MoveOut& o) {
    const int S = p.wtm ? 0 : 1;
    for (int k = 0; k < 8; ++k) {
        const int er = r + kKnightD[k][0], ec = c + kKnightD[k][1];
        if (inb(er, ec) && !((p.occ[S] >> (er * 8 + ec)) & 1)) o.add(p, r * 8 + c, er * 8 + ec, 0);
    }
}

// getKingMoves :543-573 + getCastleMoves :575-601 for the side to move. Each
// probe moves the king on the board, asks for the opponent's targets, then
// restores board[r][c] = board[end] (the king) -- literally, so a stale king
// location gets a king written to it as the reference does.
__device__ inline void king_moves(Pos& p, int r, int c, MoveOut& o) {
    const int S = p.wtm ? 0 : 1;
    const int kcode = S == 0 ? 1 : 7;
    for (int k = 0; k < 8; ++k) {
        const int er = r + kKingD[k][0], ec = c + kKingD[k][1];
        if (!inb(er, ec)) continue;
        const int dst = er * 8 + ec, src = r * 8 + c;
        if ((p.occ[S] >> dst) & 1) continue;
        const int orig = pos_at(p, dst);
        pos_set(p, src, 0);
        pos_set(p, dst, kcode);
        const bool chk = (targets(p, S ^ 1) >> dst) & 1;
        pos_set(p, src, kcode);
        pos_set(p, dst, orig);
        if (!chk) o.add(p, src, dst, 0);
    }
    // castles: squareUnderAttack on the (restored) board
    const uint64_t att = targets(p, S ^ 1);
    if ((att >> (r * 8 + c)) & 1) return;
    const int row = S == 0 ? 7 : 0;
    const int kmoved = S == 0 ? (p.flags & F_WKM) : (p.flags & F_BKM);
    if (!(p.kr[S] == row && p.kc[S] == 4) || kmoved) return;
    const uint64_t all = p.occ[0] | p.occ[1];
    const int base = row * 8;
    const int rook = S == 0 ? 3 : 9;
    const int rk = S == 0 ? (p.flags & F_WRK) : (p.flags & F_BRK);
    const int rq = S == 0 ? (p.flags & F_WRQ) : (p.flags & F_BRQ);
    if (!rk && !((all >> (base + 5)) & 1) && !((all >> (base + 6)) & 1))
        if (!((att >> (base + 5)) & 1) && !((att >> (base + 6)) & 1))
            if (pos_at(p, base + 7) == rook) o.add(p, base + 4, base + 6, MF_CASTLE);
    if (!rq && !((all >> (base + 1)) & 1) && !((all >> (base + 2)) & 1) && !((all >> (base + 3)) & 1))
        if (!((att >> (base + 2)) & 1) && !((att >> (base + 3)) & 1))
            if (pos_at(p, base + 0) == rook) o.add(p, base + 4, base + 2, MF_CASTLE);
}

__device__ inline void piece_moves(Pos& p, int t, int r, int c, MoveOut& o) {
    switch (t) {
        case 5: pawn_moves(p, r, c, nullptr, o); break;
        case 2: slide_moves(p, r, c, kRookD, o); break;
        case 4: knight_moves(p, r, c, o); break;
        case 3: slide_moves(p, r, c, kBishD, o); break;
        case 1: slide_moves(p, r, c, kRookD, o); slide_moves(p, r, c, kBishD, o); break;
        default: king_moves(p, r, c, o); break;
    }
}

struct PinList {
    int n;
    int8_t sq[8], dr[8], dc[8];
};

// getAllPossibleMoves :433-441 + addPieceMovesConsideringPins :604-630
__device__ inline void all_moves(Pos& p, const PinList& pins, MoveOut& o) {
    const int S = p.wtm ? 0 : 1;
    for (uint64_t own = p.occ[S]; own; own &= own - 1) {
        const int s = ctz64(own);
        // the board may change under king probes only at the king square itself
        const int code = pos_at(p, s);
        if (code == 0 || (code > 6 ? 1 : 0) != S) continue;
        const int t = (code - 1) % 6, r = s >> 3, c = s & 7;
        int pin = -1;
        for (int i = pins.n - 1; i >= 0; --i)
            if (pins.sq[i] == s) { pin = i; break; }
        if (pin >= 0) {
            if (t == 4) continue;
            const int pd[2] = {pins.dr[pin], pins.dc[pin]};
            const int n0 = o.n;
            if (t == 5) pawn_moves(p, r, c, pd, o);
            else piece_moves(p, t, r, c, o);
            int w = n0;
            for (int i = n0; i < o.n && i < o.cap; ++i) {
                const int to = (o.m[i] >> 6) & 63;
                const int mr = (to >> 3) - r, mc = (to & 7) - c;
                if (mr * pd[1] == mc * pd[0]) o.m[w++] = o.m[i];
            }
            o.n = w;
        } else {
            piece_moves(p, t, r, c, o);
        }
    }
}

struct CheckList {
    int n;
    int8_t r[16], c[16], dr[16], dc[16];
};

// checkForPinsAndChecks :325-383 (7 knight offsets, Q1)
__device__ inline bool pins_and_checks(const Pos& p, PinList& pins, CheckList& checks) {
    const int S = p.wtm ? 0 : 1, E = S ^ 1;
    const int kr = p.kr[S], kc = p.kc[S];
    bool in_check = false;
    pins.n = 0;
    checks.n = 0;
    for (int k = 0; k < 8; ++k) {
        const int dr = kPinD[k][0], dc = kPinD[k][1];
        int pin_sq = -1;
        for (int i = 1; i < 8; ++i) {
            const int er = kr + dr * i, ec = kc + dc * i;
            if (!inb(er, ec)) break;
            const int sq = er * 8 + ec;
            const int code = pos_at(p, sq);
            if (code == 0) continue;
            if ((code > 6 ? 1 : 0) == S) {
                if (pin_sq < 0) pin_sq = sq;
                else break;
            } else {
                const int t = (code - 1) % 6;
                const bool orth = k < 4;
                const bool hit = (orth && (t == 2 || t == 1)) || (!orth && (t == 3 || t == 1)) ||
                                 (i == 1 && t == 5 && ((E == 0 && dr == 1) || (E == 1 && dr == -1)) && !orth);
                if (hit) {
                    if (pin_sq < 0) {
                        in_check = true;
                        checks.r[checks.n] = er; checks.c[checks.n] = ec;
                        checks.dr[checks.n] = dr; checks.dc[checks.n] = dc;
                        ++checks.n;
                    } else {
                        pins.sq[pins.n] = pin_sq; pins.dr[pins.n] = dr; pins.dc[pins.n] = dc;
                        ++pins.n;
                    }
                }
                break;
            }
        }
    }
    for (int k = 0; k < 7; ++k) {
        const int er = kr + kKChkD[k][0], ec = kc + kKChkD[k][1];
        if (!inb(er, ec)) continue;
        const int code = pos_at(p, er * 8 + ec);
        if (code > 0 && (code > 6 ? 1 : 0) == E && (code - 1) % 6 == 4) {
            in_check = true;
            checks.r[checks.n] = er; checks.c[checks.n] = ec;
            checks.dr[checks.n] = kKChkD[k][0]; checks.dc[checks.n] = kKChkD[k][1];
            ++checks.n;
        }
    }
    return in_check;
}

// getValidMoves :277-321. Returns the move count (may exceed o.cap: overflow).
__device__ inline int valid_moves(Pos& p, MoveOut& o) {
    PinList pins;
    CheckList checks;
    const bool in_check = pins_and_checks(p, pins, checks);
    const int S = p.wtm ? 0 : 1;
    const int kr = p.kr[S], kc = p.kc[S];
    o.n = 0;
    o.overflow = 0;
    if (in_check) {
        if (checks.n == 1) {
            all_moves(p, pins, o);
            const int cr = checks.r[0], cc = checks.c[0];
            uint64_t valid = 0;
            const int code = pos_at(p, cr * 8 + cc);
            if (code > 0 && (code - 1) % 6 == 4) {
                valid = 1ull << (cr * 8 + cc);
            } else {
                for (int i = 1; i < 8; ++i) {
                    const int sr = kr + checks.dr[0] * i, sc = kc + checks.dc[0] * i;
                    if (inb(sr, sc)) valid |= 1ull << (sr * 8 + sc);
                    // off-board squares can never match a move's end square
                    if (sr == cr && sc == cc) break;
                }
            }
            const uint64_t att = targets(p, S ^ 1);
            int w = 0;
            const int n = o.n < o.cap ? o.n : o.cap;
            for (int i = 0; i < n; ++i) {
                const int mv = o.m[i];
                const int to = (mv >> 6) & 63;
                const bool keep = ((mv >> 12) & MF_KING) ? !((att >> to) & 1) : ((valid >> to) & 1);
                if (keep) o.m[w++] = (uint16_t)mv;
            }
            o.n = w;
        } else {
            king_moves(p, kr, kc, o);
        }
    } else {
        all_moves(p, pins, o);
    }
    return o.n;
}

// inCheck :388-394
__device__ inline bool in_check(const Pos& p) {
    const int S = p.wtm ? 0 : 1;
    const int kr = p.kr[S], kc = p.kc[S];
    if (!inb(kr, kc)) return false;
    return (targets(p, S ^ 1) >> (kr * 8 + kc)) & 1;
}

// makeMove :127-197 on a mailbox board + Pos bookkeeping fields.
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
