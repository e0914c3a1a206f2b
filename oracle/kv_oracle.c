/*
 * kv_oracle.c -- CPU restatement of the reference self-play path.
 *
 * TEST INFRASTRUCTURE ONLY. This file is the parity checker for the HIP
 * product in knightvision_amd/csrc; only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it. The product never links it.
 *
 * It restates, in plain C, with the reference's own control flow:
 *   - core/chessEngine.py GameState: getValidMoves :277-321,
 *     checkForPinsAndChecks :325-383, inCheck :388-394, squareUnderAttack
 *     :400-415, getAllPossibleMoves :433-441, piece generators :447-601,
 *     addPieceMovesConsideringPins :604-630, makeMove :127-197, isDraw :21-33,
 *     Move.__init__ :693-713 -- every quirk included.
 *   - numpy legacy RandomState: MT19937 init_genrand seeding, random_double,
 *     legacy_standard_gamma (shape < 1 branch), dirichlet (serial fp64 sum,
 *     x * (1/acc)) -- pinned numpy==1.26.0 (requirements.txt:3); the legacy
 *     stream is frozen across numpy versions.
 *   - CPython 3.10 random: init_by_array seeding, random(), choices
 *     (random.py:506-541: accumulate, total, bisect_right(cum, x, 0, n-1)),
 *     choice/_randbelow_with_getrandbits (random.py:239-249).
 *   - scripts/self_play.py _run_single_game :111-255 (buffered eval schedule,
 *     Dirichlet mixing :147-167, termination, outcome, reward) with the NN
 *     supplied by a callback.
 *
 * State vector (80 x int8, shared with tests/golden): [0..63] board codes
 * (0 empty, 1..6 wK wQ wR wB wN wp, 7..12 bK bQ bR bB bN bp; index r*8+c,
 * row 0 = rank 8), [64] whiteToMove, [65,66] whiteKingLocation, [67,68]
 * blackKingLocation, [69..74] wKingMoved bKingMoved wRookKingsideMoved
 * wRookQueensideMoved bRookKingsideMoved bRookQueensideMoved, [75,76]
 * enPassantPossible (-1 = none).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define EMPTY 0
#define WK 1
#define BK 7
#define T_K 0
#define T_Q 1
#define T_R 2
#define T_B 3
#define T_N 4
#define T_P 5
#define MAXMV 512

typedef struct {
    int8_t b[64];
    int wtm;
    int wkr, wkc, bkr, bkc;
    int wKingMoved, bKingMoved, wRK, wRQ, bRK, bRQ;
    int epr, epc;
    int inside; /* insideSquareUnderAttack :61 */
} GS;

typedef struct {
    int fr, fc, tr, tc;
    int8_t moved, captured;
    int ep, castle, promo;
} Mv;

typedef struct {
    Mv m[MAXMV];
    int n;
} ML;

/* colour char of a piece: 0 '-', 1 'w', 2 'b' */
static int colr(int p) { return p == 0 ? 0 : (p <= 6 ? 1 : 2); }
static int ptype(int p) { return (p - 1) % 6; }
static int side_col(const GS* g) { return g->wtm ? 1 : 2; }
static int enemy_col(const GS* g) { return g->wtm ? 2 : 1; }
static int inb(int r, int c) { return r >= 0 && r < 8 && c >= 0 && c < 8; }
static int at(const GS* g, int r, int c) { return g->b[r * 8 + c]; }

/* Move.__init__ :693-713 */
static void add_move(ML* l, const GS* g, int fr, int fc, int tr, int tc, int castle, int ep) {
    if (l->n >= MAXMV) abort();
    Mv* m = &l->m[l->n++];
    m->fr = fr; m->fc = fc; m->tr = tr; m->tc = tc;
    m->moved = g->b[fr * 8 + fc];
    m->captured = g->b[tr * 8 + tc];
    m->ep = ep; m->castle = castle;
    if (ep) m->captured = (m->moved == 6) ? 12 : 6; /* 'bp' if wp else 'wp' */
    m->promo = 0;
    if (m->moved != 0 && ptype(m->moved) == T_P) {
        if ((colr(m->moved) == 1 && tr == 0) || (colr(m->moved) == 2 && tr == 7)) m->promo = 1;
    }
}

static int square_under_attack(GS* g, int r, int c);

/* getPawnMoves :447-472; pin = NULL when not pinned */
static void pawn_moves(GS* g, int r, int c, ML* l, const int* pin) {
    int ma = g->wtm ? -1 : 1, start = g->wtm ? 6 : 1, enemy = enemy_col(g);
    if (!pin || (pin[0] == ma && pin[1] == 0)) {
        if (r + ma >= 0 && r + ma < 8 && at(g, r + ma, c) == EMPTY) {
            add_move(l, g, r, c, r + ma, c, 0, 0);
            if (r == start && at(g, r + 2 * ma, c) == EMPTY) add_move(l, g, r, c, r + 2 * ma, c, 0, 0);
        }
    }
    for (int k = 0; k < 2; k++) {
        int dc = k ? 1 : -1;
        if (c + dc >= 0 && c + dc < 8) {
            if (!pin || (pin[0] == ma && pin[1] == dc)) {
                if (r + ma >= 0 && r + ma < 8) {
                    if (colr(at(g, r + ma, c + dc)) == enemy)
                        add_move(l, g, r, c, r + ma, c + dc, 0, 0);
                    else if (r + ma == g->epr && c + dc == g->epc)
                        add_move(l, g, r, c, r + ma, c + dc, 0, 1);
                }
            }
        }
    }
}

static void slide(GS* g, int r, int c, ML* l, const int (*dirs)[2], int nd) {
    int enemy = enemy_col(g);
    for (int k = 0; k < nd; k++) {
        for (int i = 1; i < 8; i++) {
            int er = r + dirs[k][0] * i, ec = c + dirs[k][1] * i;
            if (!inb(er, ec)) break;
            int p = at(g, er, ec);
            if (p == EMPTY) add_move(l, g, r, c, er, ec, 0, 0);
            else if (colr(p) == enemy) { add_move(l, g, r, c, er, ec, 0, 0); break; }
            else break;
        }
    }
}

static const int ROOK_D[4][2] = {{-1, 0}, {1, 0}, {0, -1}, {0, 1}};                          /* :478 */
static const int BISH_D[4][2] = {{-1, -1}, {-1, 1}, {1, -1}, {1, 1}};                        /* :517 */
static const int KNIGHT_D[8][2] = {{-2, -1}, {-1, -2}, {-2, 1}, {-1, 2}, {1, -2}, {2, -1}, {1, 2}, {2, 1}}; /* :501 */
static const int KING_D[8][2] = {{-1, -1}, {-1, 0}, {-1, 1}, {0, -1}, {0, 1}, {1, -1}, {1, 0}, {1, 1}};    /* :544 */
static const int PIN_D[8][2] = {{-1, 0}, {0, -1}, {1, 0}, {0, 1}, {-1, -1}, {-1, 1}, {1, -1}, {1, 1}};     /* :339 */
static const int KCHK_D[7][2] = {{-2, -1}, {-1, -2}, {-1, 2}, {1, -2}, {2, -1}, {1, 2}, {2, 1}};          /* :373 (Q1) */

static void knight_moves(GS* g, int r, int c, ML* l) {
    int ally = side_col(g);
    for (int k = 0; k < 8; k++) {
        int er = r + KNIGHT_D[k][0], ec = c + KNIGHT_D[k][1];
        if (inb(er, ec)) {
            int p = at(g, er, ec);
            if (p == EMPTY || colr(p) != ally) add_move(l, g, r, c, er, ec, 0, 0);
        }
    }
}

/* getCastleMoves :575-601 */
static void castle_moves(GS* g, int r, int c, ML* l) {
    if (square_under_attack(g, r, c)) return;
    if (g->wtm) {
        if (!(g->wkr == 7 && g->wkc == 4) || g->wKingMoved) return;
        if (!g->wRK && at(g, 7, 5) == EMPTY && at(g, 7, 6) == EMPTY)
            if (!square_under_attack(g, 7, 5) && !square_under_attack(g, 7, 6))
                if (at(g, 7, 7) == 3) add_move(l, g, 7, 4, 7, 6, 1, 0);
        if (!g->wRQ && at(g, 7, 1) == EMPTY && at(g, 7, 2) == EMPTY && at(g, 7, 3) == EMPTY)
            if (!square_under_attack(g, 7, 2) && !square_under_attack(g, 7, 3))
                if (at(g, 7, 0) == 3) add_move(l, g, 7, 4, 7, 2, 1, 0);
    } else {
        if (!(g->bkr == 0 && g->bkc == 4) || g->bKingMoved) return;
        if (!g->bRK && at(g, 0, 5) == EMPTY && at(g, 0, 6) == EMPTY)
            if (!square_under_attack(g, 0, 5) && !square_under_attack(g, 0, 6))
                if (at(g, 0, 7) == 9) add_move(l, g, 0, 4, 0, 6, 1, 0);
        if (!g->bRQ && at(g, 0, 1) == EMPTY && at(g, 0, 2) == EMPTY && at(g, 0, 3) == EMPTY)
            if (!square_under_attack(g, 0, 2) && !square_under_attack(g, 0, 3))
                if (at(g, 0, 0) == 9) add_move(l, g, 0, 4, 0, 2, 1, 0);
    }
}

/* getKingMoves :543-573: each destination probed with the king moved there;
 * the restore writes board[r][c] = board[end] (the ally king), exactly as the
 * reference does, even when (r,c) is a stale king location. */
static void king_moves(GS* g, int r, int c, ML* l) {
    int ally = side_col(g);
    for (int k = 0; k < 8; k++) {
        int er = r + KING_D[k][0], ec = c + KING_D[k][1];
        if (!inb(er, ec)) continue;
        int p = at(g, er, ec);
        if (p == EMPTY || colr(p) != ally) {
            int orig = p;
            g->b[r * 8 + c] = EMPTY;
            g->b[er * 8 + ec] = g->wtm ? WK : BK;
            int okr, okc;
            if (g->wtm) { okr = g->wkr; okc = g->wkc; g->wkr = er; g->wkc = ec; }
            else { okr = g->bkr; okc = g->bkc; g->bkr = er; g->bkc = ec; }
            int chk = square_under_attack(g, er, ec);
            g->b[r * 8 + c] = g->b[er * 8 + ec];
            g->b[er * 8 + ec] = (int8_t)orig;
            if (g->wtm) { g->wkr = okr; g->wkc = okc; } else { g->bkr = okr; g->bkc = okc; }
            if (!chk) add_move(l, g, r, c, er, ec, 0, 0);
        }
    }
    castle_moves(g, r, c, l);
}

static void piece_moves(GS* g, int t, int r, int c, ML* l) {
    switch (t) {
        case T_P: pawn_moves(g, r, c, l, NULL); break;
        case T_R: slide(g, r, c, l, ROOK_D, 4); break;
        case T_N: knight_moves(g, r, c, l); break;
        case T_B: slide(g, r, c, l, BISH_D, 4); break;
        case T_Q: slide(g, r, c, l, ROOK_D, 4); slide(g, r, c, l, BISH_D, 4); break;
        case T_K: king_moves(g, r, c, l); break;
    }
}

typedef struct { int r, c, dr, dc; } Pin;

/* getAllPossibleMoves :433-441 + addPieceMovesConsideringPins :604-630 */
static void all_moves(GS* g, ML* l, const Pin* pins, int np) {
    int side = side_col(g);
    for (int r = 0; r < 8; r++)
        for (int c = 0; c < 8; c++) {
            int p = at(g, r, c);
            if (colr(p) != side) continue;
            int t = ptype(p);
            int pinned = 0, pd[2] = {0, 0};
            for (int i = np - 1; i >= 0; i--)
                if (pins[i].r == r && pins[i].c == c) { pinned = 1; pd[0] = pins[i].dr; pd[1] = pins[i].dc; break; }
            if (pinned) {
                if (t == T_N) continue;
                static ML tmp_stack[4];
                static int depth = 0; /* getKingMoves nests square_under_attack */
                ML* tmp = &tmp_stack[depth++];
                tmp->n = 0;
                if (t == T_P) pawn_moves(g, r, c, tmp, pd);
                else piece_moves(g, t, r, c, tmp);
                for (int i = 0; i < tmp->n; i++) {
                    int mr = tmp->m[i].tr - r, mc = tmp->m[i].tc - c;
                    if (mr * pd[1] == mc * pd[0]) {
                        if (l->n >= MAXMV) abort();
                        l->m[l->n++] = tmp->m[i];
                    }
                }
                depth--;
            } else {
                piece_moves(g, t, r, c, l);
            }
        }
}

/* squareUnderAttack :400-415 */
static int square_under_attack(GS* g, int r, int c) {
    if (g->inside) return 0;
    g->inside = 1;
    int orig = g->wtm;
    g->wtm = !orig;
    static ML opp;
    opp.n = 0;
    all_moves(g, &opp, NULL, 0);
    g->wtm = orig;
    g->inside = 0;
    for (int i = 0; i < opp.n; i++)
        if (opp.m[i].tr == r && opp.m[i].tc == c) return 1;
    return 0;
}

typedef struct { int r, c, dr, dc; } Chk;

/* checkForPinsAndChecks :325-383 */
static int pins_and_checks(GS* g, Pin* pins, int* np, Chk* checks, int* nc) {
    int in_check = 0;
    int enemy = enemy_col(g), ally = side_col(g);
    int kr = g->wtm ? g->wkr : g->bkr, kc = g->wtm ? g->wkc : g->bkc;
    *np = 0; *nc = 0;
    for (int k = 0; k < 8; k++) {
        int dr = PIN_D[k][0], dc = PIN_D[k][1];
        int have_pin = 0;
        Pin pp = {0, 0, 0, 0};
        for (int i = 1; i < 8; i++) {
            int er = kr + dr * i, ec = kc + dc * i;
            if (!inb(er, ec)) break;
            int p = at(g, er, ec);
            if (p == EMPTY) continue;
            if (colr(p) == ally) {
                if (!have_pin) { have_pin = 1; pp.r = er; pp.c = ec; pp.dr = dr; pp.dc = dc; }
                else break;
            } else if (colr(p) == enemy) {
                int t = ptype(p);
                int orth = (k < 4), diag = (k >= 4);
                int hit = (orth && (t == T_R || t == T_Q)) || (diag && (t == T_B || t == T_Q)) ||
                          (i == 1 && t == T_P &&
                           ((enemy == 1 && dr == 1 && (dc == -1 || dc == 1)) ||
                            (enemy == 2 && dr == -1 && (dc == -1 || dc == 1))));
                if (hit) {
                    if (!have_pin) { in_check = 1; checks[*nc] = (Chk){er, ec, dr, dc}; (*nc)++; }
                    else { pins[*np] = pp; (*np)++; }
                }
                break;
            }
        }
    }
    for (int k = 0; k < 7; k++) {
        int er = kr + KCHK_D[k][0], ec = kc + KCHK_D[k][1];
        if (inb(er, ec)) {
            int p = at(g, er, ec);
            if (colr(p) == enemy && ptype(p) == T_N) {
                in_check = 1;
                checks[*nc] = (Chk){er, ec, KCHK_D[k][0], KCHK_D[k][1]};
                (*nc)++;
            }
        }
    }
    return in_check;
}

/* getValidMoves :277-321 (checkForEndConditions :320 only sets flags) */
static void valid_moves(GS* g, ML* out) {
    Pin pins[8];
    Chk checks[16];
    int np, nc;
    int in_check = pins_and_checks(g, pins, &np, checks, &nc);
    int kr = g->wtm ? g->wkr : g->bkr, kc = g->wtm ? g->wkc : g->bkc;
    out->n = 0;
    if (in_check) {
        if (nc == 1) {
            static ML moves;
            moves.n = 0;
            all_moves(g, &moves, pins, np);
            Chk ck = checks[0];
            int vs[8][2], nv = 0;
            int piece = at(g, ck.r, ck.c);
            if (piece != EMPTY && ptype(piece) == T_N) {
                vs[0][0] = ck.r; vs[0][1] = ck.c; nv = 1;
            } else {
                for (int i = 1; i < 8; i++) {
                    int sr = kr + ck.dr * i, sc = kc + ck.dc * i;
                    vs[nv][0] = sr; vs[nv][1] = sc; nv++;
                    if (sr == ck.r && sc == ck.c) break;
                }
            }
            for (int i = 0; i < moves.n; i++) {
                Mv* m = &moves.m[i];
                if (m->moved != EMPTY && ptype(m->moved) == T_K) {
                    if (!square_under_attack(g, m->tr, m->tc)) out->m[out->n++] = *m;
                } else {
                    for (int j = 0; j < nv; j++)
                        if (vs[j][0] == m->tr && vs[j][1] == m->tc) { out->m[out->n++] = *m; break; }
                }
            }
        } else {
            king_moves(g, kr, kc, out);
        }
    } else {
        all_moves(g, out, pins, np);
    }
}

/* inCheck :388-394 */
static int in_check(GS* g) {
    return g->wtm ? square_under_attack(g, g->wkr, g->wkc) : square_under_attack(g, g->bkr, g->bkc);
}

/* makeMove :127-197 (halfMoveClock/positionCounts/FEN are inert for self-play) */
static void make_move(GS* g, const Mv* m) {
    g->b[m->fr * 8 + m->fc] = EMPTY;
    g->b[m->tr * 8 + m->tc] = m->moved;
    if (m->moved == WK) g->wKingMoved = 1;
    else if (m->moved == BK) g->bKingMoved = 1;
    else if (m->moved == 3) {
        if (m->fr == 7 && m->fc == 0) g->wRQ = 1;
        else if (m->fr == 7 && m->fc == 7) g->wRK = 1;
    } else if (m->moved == 9) {
        if (m->fr == 0 && m->fc == 0) g->bRQ = 1;
        else if (m->fr == 0 && m->fc == 7) g->bRK = 1;
    }
    if (m->ep) g->b[m->fr * 8 + m->tc] = EMPTY;
    if (m->castle) {
        if (m->tc - m->fc == 2) {
            g->b[m->tr * 8 + m->tc - 1] = g->b[m->tr * 8 + m->tc + 1];
            g->b[m->tr * 8 + m->tc + 1] = EMPTY;
        } else {
            g->b[m->tr * 8 + m->tc + 1] = g->b[m->tr * 8 + m->tc - 2];
            g->b[m->tr * 8 + m->tc - 2] = EMPTY;
        }
    }
    if (m->moved != EMPTY && ptype(m->moved) == T_P && abs(m->fr - m->tr) == 2) {
        g->epr = (m->fr + m->tr) / 2; g->epc = m->fc;
    } else {
        g->epr = g->epc = -1;
    }
    g->wtm = !g->wtm;
    if (m->moved == WK) { g->wkr = m->tr; g->wkc = m->tc; }
    else if (m->moved == BK) { g->bkr = m->tr; g->bkc = m->tc; }
    if (m->promo) g->b[m->tr * 8 + m->tc] = (int8_t)(colr(m->moved) == 1 ? 2 : 8);
}

/* GameState.isDraw :21-33 (the 50-move branch is unreachable) */
static int is_draw(const GS* g) {
    for (int i = 0; i < 64; i++)
        if (g->b[i] != EMPTY && g->b[i] != WK && g->b[i] != BK) return 0;
    return 1;
}

static void gs_from_vec(GS* g, const int8_t* v) {
    memcpy(g->b, v, 64);
    g->wtm = v[64];
    g->wkr = v[65]; g->wkc = v[66]; g->bkr = v[67]; g->bkc = v[68];
    g->wKingMoved = v[69]; g->bKingMoved = v[70];
    g->wRK = v[71]; g->wRQ = v[72]; g->bRK = v[73]; g->bRQ = v[74];
    g->epr = v[75]; g->epc = v[76];
    g->inside = 0;
}

static void gs_to_vec(const GS* g, int8_t* v) {
    memset(v, 0, 80);
    memcpy(v, g->b, 64);
    v[64] = (int8_t)g->wtm;
    v[65] = g->wkr; v[66] = g->wkc; v[67] = g->bkr; v[68] = g->bkc;
    v[69] = g->wKingMoved; v[70] = g->bKingMoved;
    v[71] = g->wRK; v[72] = g->wRQ; v[73] = g->bRK; v[74] = g->bRQ;
    v[75] = g->epr; v[76] = g->epc;
}

static void gs_init(GS* g) {
    static const int8_t start[64] = {
        9, 11, 10, 8, 7, 10, 11, 9, 12, 12, 12, 12, 12, 12, 12, 12,
        0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
        0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
        6, 6, 6, 6, 6, 6, 6, 6, 3, 5, 4, 2, 1, 4, 5, 3};
    memset(g, 0, sizeof(*g));
    memcpy(g->b, start, 64);
    g->wtm = 1;
    g->wkr = 7; g->wkc = 4; g->bkr = 0; g->bkc = 4;
    g->epr = g->epc = -1;
}

/* ------------------------------------------------------------------ API */
static void mv_pack(const Mv* m, uint8_t* o) {
    o[0] = (uint8_t)(m->fr * 8 + m->fc);
    o[1] = (uint8_t)(m->tr * 8 + m->tc);
    o[2] = (uint8_t)((m->ep ? 1 : 0) | (m->castle ? 2 : 0) | (m->promo ? 4 : 0));
}

/* getValidMoves on a state vector; the vector is updated in place (the
 * reference may mutate the board in the stale-king double-check case). */
int kvo_valid_moves(int8_t* state, uint8_t* out3, int cap) {
    GS g;
    static ML l;
    gs_from_vec(&g, state);
    valid_moves(&g, &l);
    gs_to_vec(&g, state);
    int n = l.n < cap ? l.n : cap;
    for (int i = 0; i < n; i++) mv_pack(&l.m[i], out3 + 3 * i);
    return l.n;
}

int kvo_in_check(const int8_t* state) {
    GS g;
    gs_from_vec(&g, state);
    return in_check(&g);
}

int kvo_is_draw(const int8_t* state) {
    GS g;
    gs_from_vec(&g, state);
    return is_draw(&g);
}

/* Make the index-th valid move (reference list order). Returns -1 if out of range. */
int kvo_make_valid_move(int8_t* state, int index) {
    GS g;
    static ML l;
    gs_from_vec(&g, state);
    valid_moves(&g, &l);
    if (index < 0 || index >= l.n) return -1;
    make_move(&g, &l.m[index]);
    gs_to_vec(&g, state);
    return 0;
}

void kvo_initial_state(int8_t* state) {
    GS g;
    gs_init(&g);
    gs_to_vec(&g, state);
}

/* encode_board list path ai/ai.py:17-30: planes[12][8][8] */
void kvo_encode_board(const int8_t* state, float* planes) {
    memset(planes, 0, sizeof(float) * 768);
    for (int s = 0; s < 64; s++)
        if (state[s] > 0) planes[(state[s] - 1) * 64 + s] = 1.0f;
}

/* ------------------------------------------------------------------ RNG */
typedef struct {
    uint32_t mt[624];
    int mti;
} MT;

void kvo_mt_seed_genrand(MT* s, uint32_t seed) {
    s->mt[0] = seed;
    for (int i = 1; i < 624; i++)
        s->mt[i] = 1812433253U * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
    s->mti = 624;
}

void kvo_mt_seed_by_array(MT* s, const uint32_t* key, int len) {
    kvo_mt_seed_genrand(s, 19650218U);
    int i = 1, j = 0;
    int k = 624 > len ? 624 : len;
    uint32_t* mt = s->mt;
    for (; k; k--) {
        mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525U)) + key[j] + (uint32_t)j;
        i++; j++;
        if (i >= 624) { mt[0] = mt[623]; i = 1; }
        if (j >= len) j = 0;
    }
    for (k = 623; k; k--) {
        mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941U)) - (uint32_t)i;
        i++;
        if (i >= 624) { mt[0] = mt[623]; i = 1; }
    }
    mt[0] = 0x80000000U;
}

/* CPython random.seed(int): abs value split into 32-bit little-endian words */
void kvo_mt_seed_python(MT* s, uint64_t seed) {
    uint32_t key[2];
    int n = 0;
    key[n++] = (uint32_t)seed;
    if (seed >> 32) key[n++] = (uint32_t)(seed >> 32);
    kvo_mt_seed_by_array(s, key, n);
}

uint32_t kvo_mt_next(MT* s) {
    uint32_t* mt = s->mt;
    uint32_t y;
    if (s->mti >= 624) {
        int kk;
        for (kk = 0; kk < 624 - 397; kk++) {
            y = (mt[kk] & 0x80000000U) | (mt[kk + 1] & 0x7fffffffU);
            mt[kk] = mt[kk + 397] ^ (y >> 1) ^ ((y & 1U) ? 0x9908b0dfU : 0U);
        }
        for (; kk < 623; kk++) {
            y = (mt[kk] & 0x80000000U) | (mt[kk + 1] & 0x7fffffffU);
            mt[kk] = mt[kk + (397 - 624)] ^ (y >> 1) ^ ((y & 1U) ? 0x9908b0dfU : 0U);
        }
        y = (mt[623] & 0x80000000U) | (mt[0] & 0x7fffffffU);
        mt[623] = mt[396] ^ (y >> 1) ^ ((y & 1U) ? 0x9908b0dfU : 0U);
        s->mti = 0;
    }
    y = mt[s->mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680U;
    y ^= (y << 15) & 0xefc60000U;
    y ^= (y >> 18);
    return y;
}

double kvo_res53(MT* s) {
    uint32_t a = kvo_mt_next(s) >> 5, b = kvo_mt_next(s) >> 6;
    return (a * 67108864.0 + b) / 9007199254740992.0;
}

/* numpy legacy_standard_gamma, shape in (0,1) (shape==1 / >1 branches are not
 * reachable with DIR_NOISE_ALPHA < 1; the caller asserts). Each attempt reads
 * exactly 4 u32: U = res53, V = -log(1 - res53). */
static double legacy_gamma_small(MT* s, double shape, uint64_t* attempts) {
    for (;;) {
        double U = kvo_res53(s);
        double V = -log(1.0 - kvo_res53(s));
        (*attempts)++;
        if (U <= 1.0 - shape) {
            double X = pow(U, 1. / shape);
            if (X <= V) return X;
        } else {
            double Y = -log((1 - U) / shape);
            double X = pow(1.0 - shape + shape * Y, 1. / shape);
            if (X <= (V + Y)) return X;
        }
    }
}

/* RandomState.dirichlet([alpha]*k) legacy: gamma draws, serial acc, x*(1/acc).
 * Returns the number of gamma attempts (u32 consumed = 4 * attempts). */
int64_t kvo_dirichlet(MT* s, double alpha, int k, double* out) {
    if (!(alpha > 0.0 && alpha < 1.0)) return -1;
    uint64_t attempts = 0;
    double acc = 0.0;
    for (int j = 0; j < k; j++) {
        out[j] = legacy_gamma_small(s, alpha, &attempts);
        acc = acc + out[j];
    }
    double invacc = 1 / acc;
    for (int j = 0; j < k; j++) out[j] = out[j] * invacc;
    return (int64_t)attempts;
}

/* random.choices(population, weights, k=1) -> index (CPython 3.10 random.py:506-541) */
int kvo_choices(MT* s, const double* w, int n) {
    double cum = 0.0;
    double* cw = (double*)malloc(sizeof(double) * (size_t)n);
    for (int i = 0; i < n; i++) { cum = cum + w[i]; cw[i] = cum; }
    double total = cw[n - 1] + 0.0;
    double x = kvo_res53(s) * total;
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        int mid = (lo + hi) / 2;
        if (x < cw[mid]) hi = mid; else lo = mid + 1;
    }
    free(cw);
    return lo;
}

/* random.choice -> _randbelow_with_getrandbits(n), random.py:239-249 */
int kvo_randbelow(MT* s, int n) {
    int k = 0;
    while ((n >> k) != 0) k++; /* n.bit_length() */
    uint32_t r = kvo_mt_next(s) >> (32 - k);
    while ((int)r >= n) r = kvo_mt_next(s) >> (32 - k);
    return (int)r;
}

/* torch.softmax(float32) restated: max, exp(x - max), sum, x * (1/sum) */
void kvo_softmax_f32(const float* x, int n, float* y) {
    float m = x[0];
    for (int i = 1; i < n; i++) m = x[i] > m ? x[i] : m;
    float s = 0.0f;
    for (int i = 0; i < n; i++) { y[i] = expf(x[i] - m); s += y[i]; }
    float inv = 1.0f / s;
    for (int i = 0; i < n; i++) y[i] = y[i] * inv;
}

/* ------------------------------------------------------------ self-play */
typedef void (*kvo_eval_fn)(void* ctx, const float* planes, int n, float* logits, float* values);
typedef void (*kvo_softmax_fn)(void* ctx, const float* logits, float* probs);

typedef struct {
    float logits[4096];
    float value;
    int has;
} kvo_last;

typedef struct {
    int max_moves;     /* <= 0: None */
    int batch;         /* SELFPLAY_BATCH_SIZE */
    double eps, alpha; /* DIR_NOISE_EPS, DIR_NOISE_ALPHA */
} kvo_game_cfg;

typedef struct {
    int plies;
    int outcome;      /* +1 / 0 / -1 */
    float reward;     /* 1.0 / 0.2 / -1.0 */
    int reason;       /* 0 max_moves 1 resign 2 mate 3 stalemate 4 draw 5 material */
    int n_evals;      /* forward calls */
} kvo_game_result;

static void eval_buffer(kvo_eval_fn cb, void* ctx, float* buf, int n, kvo_last* last, int* sizes, int* nsz) {
    static float* lg = NULL;
    static float* vl = NULL;
    static int capn = 0;
    if (n > capn) {
        free(lg); free(vl);
        lg = (float*)malloc(sizeof(float) * 4096 * (size_t)n);
        vl = (float*)malloc(sizeof(float) * (size_t)n);
        capn = n;
    }
    cb(ctx, buf, n, lg, vl);
    memcpy(last->logits, lg + (size_t)(n - 1) * 4096, sizeof(float) * 4096);
    last->value = vl[n - 1];
    last->has = 1;
    if (sizes) sizes[(*nsz)++] = n;
}

/* _run_single_game :111-255. np_mt / py_mt are the numpy and CPython streams;
 * `last` is the function attribute _run_single_game._last_outputs. Records:
 * states (80 B each) and move indices; returns plies. */
int kvo_play_game(const kvo_game_cfg* cfg, MT* np_mt, MT* py_mt, kvo_eval_fn cb, kvo_softmax_fn smx, void* ctx,
                  kvo_last* last, int8_t* rec_states, uint16_t* rec_moves, int cap, int* eval_sizes, int size_cap,
                  kvo_game_result* res) {
    GS g;
    gs_init(&g);
    static ML ml;
    float* buf = (float*)malloc(sizeof(float) * 768 * (size_t)(cfg->batch > 0 ? cfg->batch : 1));
    float probs[4096];
    double* noise = (double*)malloc(sizeof(double) * 4096);
    double* legal = (double*)malloc(sizeof(double) * MAXMV);
    int nbuf = 0, move_count = 0, maxed = 0, resigned = 0, outcome = 0, reason = -1, nsz = 0;
    int8_t vec[80];
    (void)size_cap;
    for (;;) {
        valid_moves(&g, &ml);
        if (ml.n == 0) break;
        gs_to_vec(&g, vec);
        kvo_encode_board(vec, buf + (size_t)nbuf * 768);
        nbuf++;
        if (nbuf >= cfg->batch) { eval_buffer(cb, ctx, buf, nbuf, last, eval_sizes, &nsz); nbuf = 0; }
        if (!last->has) { eval_buffer(cb, ctx, buf, nbuf, last, eval_sizes, &nsz); nbuf = 0; }
        if (smx) smx(ctx, last->logits, probs);
        else kvo_softmax_f32(last->logits, 4096, probs);
        kvo_dirichlet(np_mt, cfg->alpha, 4096, noise);
        float keep = (float)(1.0 - cfg->eps);
        double total = 0.0;
        for (int i = 0; i < ml.n; i++) {
            int idx = (ml.m[i].fr * 8 + ml.m[i].fc) * 64 + ml.m[i].tr * 8 + ml.m[i].tc;
            float p32 = keep * probs[idx];
            legal[i] = (double)p32 + cfg->eps * noise[idx];
            total = total + legal[i];
        }
        int pick;
        if (total == 0.0) {
            pick = kvo_randbelow(py_mt, ml.n);
        } else {
            for (int i = 0; i < ml.n; i++) legal[i] = legal[i] / total;
            pick = kvo_choices(py_mt, legal, ml.n);
        }
        const Mv* m = &ml.m[pick];
        if (move_count < cap) {
            if (rec_states) memcpy(rec_states + (size_t)move_count * 80, vec, 80);
            rec_moves[move_count] = (uint16_t)((m->fr * 8 + m->fc) * 64 + m->tr * 8 + m->tc);
        }
        make_move(&g, m);
        move_count++;
        if (is_draw(&g)) break;
        if (move_count > 15 && (double)last->value < -0.7) {
            outcome = g.wtm ? -1 : 1;
            reason = 1;
            resigned = 1;
            break;
        }
        if (cfg->max_moves > 0 && move_count >= cfg->max_moves) { maxed = 1; break; }
    }
    if (nbuf) { eval_buffer(cb, ctx, buf, nbuf, last, eval_sizes, &nsz); nbuf = 0; }
    if (maxed) { outcome = 0; reason = 0; }
    else if (resigned) { /* set above */ }
    else {
        int chk = in_check(&g);
        valid_moves(&g, &ml);
        int n1 = ml.n;
        if (chk && n1 == 0) { outcome = g.wtm ? -1 : 1; reason = 2; }
        else {
            valid_moves(&g, &ml);
            if (ml.n == 0) { outcome = 0; reason = 3; }
            else if (is_draw(&g)) { outcome = 0; reason = 4; }
            else {
                /* material branch :229-238 restated literally: the codes are
                 * two-char strings, so 'wX'.isupper() is never true and
                 * piece_value('wp'.upper() == 'WP') is 0 -- both sums are 0 and
                 * the outcome is always 0. */
                outcome = 0;
                reason = 5;
            }
        }
    }
    res->plies = move_count;
    res->outcome = outcome;
    res->reward = outcome == 1 ? 1.0f : (outcome == 0 ? 0.2f : -1.0f);
    res->reason = reason;
    res->n_evals = nsz;
    free(buf); free(noise); free(legal);
    return move_count;
}

/* expose struct sizes so the ctypes wrapper can allocate opaque blobs */
int kvo_sizeof_mt(void) { return (int)sizeof(MT); }
int kvo_sizeof_last(void) { return (int)sizeof(kvo_last); }

/* ----------------------------------------------------------- MCTS ------
 * CPU restatement of the build-defined PUCT search of
 * knightvision_amd/csrc/kv_mcts.hip (no reference counterpart). Same
 * capacities, same fp32 operation order (-ffp-contract=off), same RNG use:
 * the root priors are the reference's mixed legal weights (self_play.py
 * :147-166) normalised, the move is random.choices over root visit counts.
 * The root softmax and the leaf priors (legal moves' logits only) use
 * kvo_det_expf and the device's lane / butterfly summation order, so every
 * prior equals the device's bit for bit given the same network rows.
 * eval_cb == NULL selects the hash test evaluator (all logits 0, value =
 * dyadic FNV-1a hash of the 64 board codes), which is exact on both sides. */
typedef struct {
    int sims;
    float c_puct;
    int max_moves;
    double eps, alpha;
    int edge_cap; /* <= 0: KV_MAXM x (sims + 1) (kv_engine.hip kv_create), which cannot overflow */
} kvo_mcts_cfg;

#define KVO_MAXM 320 /* include/kv.h KV_MAXM */

/* det_expf of kv_engine.h: exp from IEEE double basic operations (this file
 * is compiled with -ffp-contract=off), Cody-Waite by ln 2, degree-11 Taylor,
 * exact 2^k scaling, one rounding to float; 0 below e^-87. */
float kvo_det_expf(float x) {
    if (!(x >= -87.0f)) return 0.0f;
    const double xd = (double)x;
    const double kd = rint(xd * 1.4426950408889634);
    const double r = (xd - kd * 6.93147180369123816490e-01) - kd * 1.90821492927058770002e-10;
    double p = 2.5052108385441720e-08;
    p = p * r + 2.7557319223985893e-07;
    p = p * r + 2.7557319223985888e-06;
    p = p * r + 2.4801587301587302e-05;
    p = p * r + 1.9841269841269841e-04;
    p = p * r + 1.3888888888888889e-03;
    p = p * r + 8.3333333333333332e-03;
    p = p * r + 4.1666666666666664e-02;
    p = p * r + 1.6666666666666666e-01;
    p = p * r + 0.5;
    p = p * r + 1.0;
    p = p * r + 1.0;
    const uint64_t bits = (uint64_t)((int64_t)kd + 1023) << 52;
    double scale;
    memcpy(&scale, &bits, sizeof scale);
    return (float)(p * scale);
}

/* the wave's xor-butterfly sum (kv_engine.h wave_sum) over 64 lane partials */
static float wave_sum64(float* part) {
    float t[64];
    for (int m = 32; m >= 1; m >>= 1) {
        for (int l = 0; l < 64; ++l) t[l] = part[l] + part[l ^ m];
        memcpy(part, t, sizeof t);
    }
    return part[0];
}

/* kv_engine.h wave_softmax_4096_det: lane l holds entries j*64+l, j = 0..63 */
void kvo_softmax_det_4096(const float* lg, float* out) {
    float m = -INFINITY;
    for (int i = 0; i < 4096; ++i) m = fmaxf(m, lg[i]);
    float part[64];
    static float e[4096];
    for (int l = 0; l < 64; ++l) {
        float s = 0.f;
        for (int j = 0; j < 64; ++j) {
            e[j * 64 + l] = kvo_det_expf(lg[j * 64 + l] - m);
            s += e[j * 64 + l];
        }
        part[l] = s;
    }
    const float inv = 1.0f / wave_sum64(part);
    for (int i = 0; i < 4096; ++i) out[i] = e[i] * inv;
}

/* kv_mcts.hip leaf priors: softmax over the n legal moves' logits; lane l
 * sums entries l, l+64, ... in order, then the butterfly. e[] receives the
 * unnormalised terms; returns the sum. */
static float legal_softmax_terms(const float* lg, const int* idx, int n, float* e) {
    float mx = -INFINITY;
    for (int j = 0; j < n; ++j) mx = fmaxf(mx, lg[idx[j]]);
    float part[64];
    for (int l = 0; l < 64; ++l) {
        float s = 0.f;
        for (int j = l; j < n; j += 64) {
            e[j] = kvo_det_expf(lg[idx[j]] - mx);
            s += e[j];
        }
        part[l] = s;
    }
    return wave_sum64(part);
}

static void hash_eval_board(const int8_t* b, float* logits, float* value) {
    uint32_t h = 2166136261u;
    for (int q = 0; q < 64; ++q) { h ^= (uint8_t)b[q]; h *= 16777619u; }
    for (int j = 0; j < 4096; ++j) logits[j] = 0.f;
    *value = (float)((int)(h % 129u) - 64) / 64.0f;
}


static float puct_score(float c_puct, float P, float sq, int N, float W) {
    const float u = c_puct * P * sq / (float)(1 + N);
    const float q = N > 0 ? W / (float)N : 0.0f;
    return q + u;
}

static int choose_weighted_c(MT* py, const double* w, int n) {
    double total = 0.0;
    for (int j = 0; j < n; ++j) total = total + w[j];
    if (total == 0.0) return kvo_randbelow(py, n);
    double* nw = (double*)malloc(sizeof(double) * (size_t)n);
    for (int j = 0; j < n; ++j) nw[j] = w[j] / total;
    int k = kvo_choices(py, nw, n);
    free(nw);
    return k;
}

/* One game's search state (the lock-step batch below plays G of them; the
 * single game is the batch of one, so both give the same bits per game). */
typedef struct {
    const kvo_mcts_cfg* cfg;
    MT *np_mt, *py_mt;
    int S, ncap, ecap, overflow;
    float* sqt;
    Mv* e_mv;
    float *e_P, *e_W;
    int *e_N, *e_child, *n_first, *n_cnt, *n_N, *path;
    float *logits, *probs, *lterm;
    double *noise, *w;
    int* lidx;
    ML *ml, *lm;
    GS g, b;
    int move_count, outcome, reason, maxed, resigned, evals, done;
    float root_value, v;
    int root_wtm, node_count, edge_count, depth, leaf;
    uint16_t* rec_moves;
    int cap;
    int32_t* visits;
    int maxm;
} MG;

static void mg_init(MG* m, const kvo_mcts_cfg* cfg, MT* np_mt, MT* py_mt, uint16_t* rec_moves, int cap,
                    int32_t* visits, int maxm) {
    memset(m, 0, sizeof *m);
    m->cfg = cfg; m->np_mt = np_mt; m->py_mt = py_mt;
    m->S = cfg->sims; m->ncap = m->S + 2;
    const int full = KVO_MAXM * (m->S + 1);
    m->ecap = cfg->edge_cap > 0 && cfg->edge_cap < full ? cfg->edge_cap : full;
    m->sqt = (float*)malloc(sizeof(float) * (size_t)(m->ncap + 2));
    for (int k = 0; k < m->ncap + 2; ++k) m->sqt[k] = (float)sqrt((double)k);
    m->e_mv = (Mv*)malloc(sizeof(Mv) * (size_t)m->ecap);
    m->e_P = (float*)malloc(sizeof(float) * (size_t)m->ecap);
    m->e_N = (int*)malloc(sizeof(int) * (size_t)m->ecap);
    m->e_W = (float*)malloc(sizeof(float) * (size_t)m->ecap);
    m->e_child = (int*)malloc(sizeof(int) * (size_t)m->ecap);
    m->n_first = (int*)malloc(sizeof(int) * (size_t)m->ncap);
    m->n_cnt = (int*)malloc(sizeof(int) * (size_t)m->ncap);
    m->n_N = (int*)malloc(sizeof(int) * (size_t)m->ncap);
    m->path = (int*)malloc(sizeof(int) * (size_t)m->ncap);
    m->logits = (float*)malloc(sizeof(float) * 4096);
    m->probs = (float*)malloc(sizeof(float) * 4096);
    m->noise = (double*)malloc(sizeof(double) * 4096);
    m->w = (double*)malloc(sizeof(double) * MAXMV);
    m->lidx = (int*)malloc(sizeof(int) * MAXMV);
    m->lterm = (float*)malloc(sizeof(float) * MAXMV);
    m->ml = (ML*)malloc(sizeof(ML));
    m->lm = (ML*)malloc(sizeof(ML));
    m->reason = -1;
    m->rec_moves = rec_moves; m->cap = cap; m->visits = visits; m->maxm = maxm;
    gs_init(&m->g);
}

static void mg_free(MG* m) {
    free(m->sqt); free(m->e_mv); free(m->e_P); free(m->e_N); free(m->e_W); free(m->e_child); free(m->n_first);
    free(m->n_cnt); free(m->n_N); free(m->path); free(m->logits); free(m->probs); free(m->noise); free(m->w);
    free(m->lidx); free(m->lterm); free(m->ml); free(m->lm);
}

/* start of a move: 1 = the root position needs a network row, 0 = the game is over (no legal move) */
static int mg_move_start(MG* m) {
    valid_moves(&m->g, m->ml);
    if (m->ml->n == 0) { m->done = 1; return 0; }
    return 1;
}

/* the root's network row (logits in m->logits, value) -> priors and a fresh tree */
static void mg_root(MG* m, float root_value) {
    const kvo_mcts_cfg* cfg = m->cfg;
    const ML* ml = m->ml;
    m->root_value = root_value;
    m->evals++;
    kvo_softmax_det_4096(m->logits, m->probs);
    kvo_dirichlet(m->np_mt, cfg->alpha, 4096, m->noise);
    const float keep = (float)(1.0 - cfg->eps);
    double total = 0.0;
    for (int i = 0; i < ml->n; i++) {
        int idx = (ml->m[i].fr * 8 + ml->m[i].fc) * 64 + ml->m[i].tr * 8 + ml->m[i].tc;
        float p32 = keep * m->probs[idx];
        m->w[i] = (double)p32 + cfg->eps * m->noise[idx];
        total = total + m->w[i];
    }
    m->root_wtm = m->g.wtm;
    m->node_count = 1;
    m->edge_count = ml->n;
    m->n_first[0] = 0; m->n_cnt[0] = ml->n; m->n_N[0] = 1;
    for (int i = 0; i < ml->n; i++) {
        m->e_mv[i] = ml->m[i];
        m->e_P[i] = total == 0.0 ? 1.0f / (float)ml->n : (float)(m->w[i] / total);
        m->e_N[i] = 0; m->e_W[i] = 0.f; m->e_child[i] = -1;
    }
}

/* one simulation's descent: 1 = the leaf position (m->b) needs a network row,
 * 0 = its value is known (draw, mate, stalemate; m->v) */
static int mg_descend(MG* m) {
    m->b = m->g;
    int node = 0;
    m->depth = 0;
    m->leaf = -1;
    for (;;) {
        const int first = m->n_first[node], cnt = m->n_cnt[node];
        const float sq = m->sqt[m->n_N[node]];
        float best = -INFINITY;
        int bi = 0;
        for (int j = 0; j < cnt; ++j) {
            const float sc = puct_score(m->cfg->c_puct, m->e_P[first + j], sq, m->e_N[first + j], m->e_W[first + j]);
            if (sc > best) { best = sc; bi = j; }
        }
        const int e = first + bi;
        m->path[m->depth++] = e;
        make_move(&m->b, &m->e_mv[e]);
        const int child = m->e_child[e];
        if (child < 0 || m->depth >= m->ncap) { m->leaf = e; break; }
        node = child;
    }
    m->v = 0.f;
    if (is_draw(&m->b)) return 0;
    valid_moves(&m->b, m->lm);
    if (m->lm->n == 0) {
        m->v = in_check(&m->b) ? (m->b.wtm ? -1.f : 1.f) : 0.f;
        return 0;
    }
    return 1;
}

/* the leaf's network row (m->logits, value) -> expansion */
static void mg_expand(MG* m, float value) {
    const ML* lm = m->lm;
    m->v = value;
    m->evals++;
    for (int j = 0; j < lm->n; ++j)
        m->lidx[j] = (lm->m[j].fr * 8 + lm->m[j].fc) * 64 + lm->m[j].tr * 8 + lm->m[j].tc;
    const float sum = legal_softmax_terms(m->logits, m->lidx, lm->n, m->lterm);
    if (m->edge_count + lm->n <= m->ecap && m->node_count < m->ncap) {
        const int id = m->node_count++;
        m->n_first[id] = m->edge_count; m->n_cnt[id] = lm->n; m->n_N[id] = 0;
        for (int j = 0; j < lm->n; ++j) {
            const int e = m->edge_count + j;
            m->e_mv[e] = lm->m[j];
            m->e_P[e] = sum > 0.f ? m->lterm[j] / sum : 1.0f / (float)lm->n;
            m->e_N[e] = 0; m->e_W[e] = 0.f; m->e_child[e] = -1;
        }
        m->edge_count += lm->n;
        m->e_child[m->leaf] = id;
    } else {
        m->overflow++;
    }
}

static void mg_backup(MG* m) {
    m->n_N[0] += 1;
    for (int d = 0; d < m->depth; ++d) {
        const int e = m->path[d];
        const int white_moved = ((m->root_wtm != 0) ^ (d & 1)) != 0;
        m->e_N[e] += 1;
        m->e_W[e] = m->e_W[e] + (white_moved ? m->v : -m->v);
        const int nd = m->e_child[e];
        if (nd >= 0) m->n_N[nd] += 1;
    }
}

/* the move: random.choices over the root visit counts, then the reference's termination checks */
static void mg_commit(MG* m) {
    const ML* ml = m->ml;
    for (int i = 0; i < ml->n; ++i) m->w[i] = (double)m->e_N[i];
    if (m->visits && m->move_count < m->cap)
        for (int j = 0; j < m->maxm; ++j)
            m->visits[(size_t)m->move_count * m->maxm + j] = j < ml->n ? m->e_N[j] : -1;
    const int pick = choose_weighted_c(m->py_mt, m->w, ml->n);
    const Mv mv = ml->m[pick];
    if (m->move_count < m->cap) m->rec_moves[m->move_count] = (uint16_t)((mv.fr * 8 + mv.fc) * 64 + mv.tr * 8 + mv.tc);
    make_move(&m->g, &mv);
    m->move_count++;
    if (is_draw(&m->g)) { m->done = 1; return; }
    if (m->move_count > 15 && (double)m->root_value < -0.7) {
        m->outcome = m->g.wtm ? -1 : 1; m->reason = 1; m->resigned = 1; m->done = 1; return;
    }
    if (m->cfg->max_moves > 0 && m->move_count >= m->cfg->max_moves) { m->maxed = 1; m->done = 1; }
}

static void mg_result(MG* m, kvo_game_result* res) {
    GS* g = &m->g;
    if (m->maxed) { m->outcome = 0; m->reason = 0; }
    else if (!m->resigned) {
        int chk = in_check(g);
        int mate = 0;
        if (chk) { valid_moves(g, m->ml); mate = m->ml->n == 0; }
        if (mate) { m->outcome = g->wtm ? -1 : 1; m->reason = 2; }
        else {
            valid_moves(g, m->ml);
            if (m->ml->n == 0) { m->outcome = 0; m->reason = 3; }
            else { m->outcome = 0; m->reason = is_draw(g) ? 4 : 5; }
        }
    }
    res->plies = m->move_count;
    res->outcome = m->outcome;
    res->reward = m->outcome == 1 ? 1.0f : (m->outcome == 0 ? 0.2f : -1.0f);
    res->reason = m->reason;
    res->n_evals = m->evals;
}

/* network rows of the games in want[] (positions gs[k]): one callback over all of them (the
 * leaf batch), or the hash test evaluator per game; results into each game's m->logits, val[k] */
static void mg_eval(MG* const* want, const GS* const* pos, int n, kvo_eval_fn cb, void* ctx, float* planes,
                    float* lg, float* val) {
    if (!cb) {
        for (int k = 0; k < n; ++k) hash_eval_board(pos[k]->b, want[k]->logits, &val[k]);
        return;
    }
    int8_t vec[80];
    for (int k = 0; k < n; ++k) {
        gs_to_vec(pos[k], vec);
        kvo_encode_board(vec, planes + (size_t)k * 768);
    }
    cb(ctx, planes, n, lg, val);
    for (int k = 0; k < n; ++k) memcpy(want[k]->logits, lg + (size_t)k * 4096, sizeof(float) * 4096);
}

/* G games in lock-step (the device's batch shape: every game runs the same
 * simulation index, the leaves that need the network go out as one batch of
 * up to G rows). Game k uses np_mts[k] / py_mts[k], records rec_moves + k*cap
 * and (visits != NULL) visits + k*cap*maxm, and res[k]. Each game's search is
 * the single-game one exactly (the batch only groups the network calls).
 * Returns 0, or -1 when some expansion did not fit its edge pool. */
int kvo_mcts_play_batch(const kvo_mcts_cfg* cfg, int G, MT** np_mts, MT** py_mts, kvo_eval_fn cb, void* ctx,
                        uint16_t* rec_moves, int cap, int32_t* visits, int maxm, kvo_game_result* res) {
    MG* gm = (MG*)malloc(sizeof(MG) * (size_t)G);
    MG** want = (MG**)malloc(sizeof(MG*) * (size_t)G);
    const GS** pos = (const GS**)malloc(sizeof(GS*) * (size_t)G);
    float* planes = (float*)malloc(sizeof(float) * 768 * (size_t)G);
    float* lg = (float*)malloc(sizeof(float) * 4096 * (size_t)G);
    float* val = (float*)malloc(sizeof(float) * (size_t)G);
    for (int k = 0; k < G; ++k)
        mg_init(&gm[k], cfg, np_mts[k], py_mts[k], rec_moves + (size_t)k * cap, cap,
                visits ? visits + (size_t)k * cap * maxm : NULL, maxm);
    for (;;) {
        int n = 0;
        for (int k = 0; k < G; ++k)
            if (!gm[k].done && mg_move_start(&gm[k])) { want[n] = &gm[k]; pos[n] = &gm[k].g; n++; }
        if (n == 0) break;
        mg_eval(want, pos, n, cb, ctx, planes, lg, val);
        for (int k = 0; k < n; ++k) mg_root(want[k], val[k]);
        MG** act = (MG**)malloc(sizeof(MG*) * (size_t)n);
        const int na = n;
        memcpy(act, want, sizeof(MG*) * (size_t)na);
        for (int s = 0; s < cfg->sims; ++s) {
            n = 0;
            for (int k = 0; k < na; ++k)
                if (mg_descend(act[k])) { want[n] = act[k]; pos[n] = &act[k]->b; n++; }
            if (n) mg_eval(want, pos, n, cb, ctx, planes, lg, val);
            for (int k = 0; k < n; ++k) mg_expand(want[k], val[k]);
            for (int k = 0; k < na; ++k) mg_backup(act[k]);
        }
        for (int k = 0; k < na; ++k) mg_commit(act[k]);
        free(act);
    }
    int overflow = 0;
    for (int k = 0; k < G; ++k) {
        mg_result(&gm[k], &res[k]);
        overflow |= gm[k].overflow != 0;
        mg_free(&gm[k]);
    }
    free(gm); free(want); free(pos); free(planes); free(lg); free(val);
    return overflow ? -1 : 0;
}

/* plays one game; rec_moves[ply], visits[ply * maxm + j] = root visit counts
 * in root move-list order (maxm entries per ply, -1 padded). Returns the
 * number of plies, or -1 when an expansion did not fit the edge pool (the
 * device raises KV_EOVERFLOW there). */
int kvo_mcts_play_game(const kvo_mcts_cfg* cfg, MT* np_mt, MT* py_mt, kvo_eval_fn cb, void* ctx,
                       uint16_t* rec_moves, int cap, int32_t* visits, int maxm, kvo_game_result* res) {
    const int rc = kvo_mcts_play_batch(cfg, 1, &np_mt, &py_mt, cb, ctx, rec_moves, cap, visits, maxm, res);
    return rc < 0 ? -1 : res->plies;
}
