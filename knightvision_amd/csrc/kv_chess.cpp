// Full-rules chess for the reference's data pipeline (host code in libkv.so).
//
// The reference's PGN -> JSONL ingestion (data_utils/parser_pgn.py:81-185)
// and its two JSONL datasets (data_utils/dataset.py:29-91, ChessDataset;
// scripts/train.py:497-561, ChessPGNDataset) run on python-chess 1.999
// (requirements.txt:5), which is not installed here. This file restates the
// parts of python-chess they use, with python-chess's square numbering
// (a1 = 0, h8 = 63) and its conventions:
//   * Board(fen) / Board.fen(): en-passant square printed only when a legal
//     en-passant capture exists ("legal" mode), castling rights cleaned to
//     rooks / kings still on their original squares, "KQkq" order;
//   * Board.push(): ep square after every double push, halfmove clock reset on
//     pawn moves and captures, castling rights cleared by any move from / to
//     a king or corner-rook square;
//   * Board.san(): piece letter, file / rank disambiguation against the other
//     legal moves of the same piece type to the same square (file first, rank
//     when the file is shared), pawn captures with the from-file, "x", "=Q"
//     promotions, "O-O" / "O-O-O", "+" / "#" suffixes;
//   * Board.parse_san(): the SAN regex ^([NBKRQ])?([a-h])?([1-8])?[-x]?
//     ([a-h][1-8])(=?[nbrqkNBRQK])?[+#]?$, castling spellings with O or 0,
//     null moves "--" / "Z0" / "0000" / "@@@@", pawn moves restricted to the
//     target file unless a from-file is given, ambiguity and illegality errors;
//   * chess.pgn.read_game(): tag pairs, "%" / ";" lines, {} comments (multi-
//     line), ";" comments, NAGs, "?!" glyphs, variations (skipped: they do
//     not change the mainline), move numbers, the result token (sets a "*"
//     Result header), a blank line ends the movetext, the first illegal or
//     unparsable mainline SAN ends the game's mainline (game.errors), and the
//     FEN tag sets the start position.
// Legality is make-and-test (king not attacked after the move); perft counts
// of the standard test positions pin it (tests/test_chess_cpu.py).
#include <ctype.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/kv.h"

namespace kv {
void set_error(const char* fmt, ...);
}

namespace {

enum { EMPTY = 0, PAWN = 1, KNIGHT = 2, BISHOP = 3, ROOK = 4, QUEEN = 5, KING = 6 };
// piece code: 0 empty, 1..6 white P N B R Q K, 7..12 black p n b r q k
inline int ptype(int pc) { return pc == 0 ? 0 : (pc - 1) % 6 + 1; }
inline bool pwhite(int pc) { return pc >= 1 && pc <= 6; }
inline int mkpc(int type, bool white) { return white ? type : type + 6; }
inline int file_of(int s) { return s & 7; }
inline int rank_of(int s) { return s >> 3; }
const char PIECE_CHARS[] = ".PNBRQKpnbrqk";

enum { CR_WK = 1, CR_WQ = 2, CR_BK = 4, CR_BQ = 8 };

struct Move {
    int from = 0, to = 0, promo = 0;  // promo: piece type or 0
    bool null() const { return from == to; }
};

struct Board {
    int8_t sq[64];
    bool white = true;
    int castle = 0;
    int ep = -1;  // after a double push (python-chess Board.ep_square), printed only when capturable
    int halfmove = 0, fullmove = 1;
};

const int KN_D[8][2] = {{1, 2}, {2, 1}, {2, -1}, {1, -2}, {-1, -2}, {-2, -1}, {-2, 1}, {-1, 2}};
const int KG_D[8][2] = {{1, 0}, {1, 1}, {0, 1}, {-1, 1}, {-1, 0}, {-1, -1}, {0, -1}, {1, -1}};
const int RK_D[4][2] = {{1, 0}, {-1, 0}, {0, 1}, {0, -1}};
const int BS_D[4][2] = {{1, 1}, {1, -1}, {-1, 1}, {-1, -1}};

inline bool on(int f, int r) { return f >= 0 && f < 8 && r >= 0 && r < 8; }

// is square s attacked by side `by_white`
bool attacked(const Board& b, int s, bool by_white) {
    const int f = file_of(s), r = rank_of(s);
    const int pr = by_white ? r - 1 : r + 1;  // rank the attacking pawn stands on
    for (int df = -1; df <= 1; df += 2)
        if (on(f + df, pr) && b.sq[pr * 8 + f + df] == mkpc(PAWN, by_white)) return true;
    for (auto& d : KN_D)
        if (on(f + d[0], r + d[1]) && b.sq[(r + d[1]) * 8 + f + d[0]] == mkpc(KNIGHT, by_white)) return true;
    for (auto& d : KG_D)
        if (on(f + d[0], r + d[1]) && b.sq[(r + d[1]) * 8 + f + d[0]] == mkpc(KING, by_white)) return true;
    for (int k = 0; k < 2; ++k) {
        const int(*D)[2] = k == 0 ? RK_D : BS_D;
        const int slider = k == 0 ? ROOK : BISHOP;
        for (int i = 0; i < 4; ++i) {
            int ff = f + D[i][0], rr = r + D[i][1];
            while (on(ff, rr)) {
                const int pc = b.sq[rr * 8 + ff];
                if (pc) {
                    if (pwhite(pc) == by_white && (ptype(pc) == slider || ptype(pc) == QUEEN)) return true;
                    break;
                }
                ff += D[i][0];
                rr += D[i][1];
            }
        }
    }
    return false;
}

int king_sq(const Board& b, bool white) {
    for (int s = 0; s < 64; ++s)
        if (b.sq[s] == mkpc(KING, white)) return s;
    return -1;
}

bool in_check(const Board& b) {
    const int k = king_sq(b, b.white);
    return k >= 0 && attacked(b, k, !b.white);
}

bool is_ep_capture(const Board& b, const Move& m) {
    return ptype(b.sq[m.from]) == PAWN && m.to == b.ep && file_of(m.from) != file_of(m.to) && b.sq[m.to] == 0;
}

bool is_castling(const Board& b, const Move& m) {
    return ptype(b.sq[m.from]) == KING && abs(file_of(m.to) - file_of(m.from)) == 2;
}

bool is_capture(const Board& b, const Move& m) {
    const int t = b.sq[m.to];
    return (t && pwhite(t) != b.white) || is_ep_capture(b, m);
}

// python-chess Board.push (standard chess)
void push(Board& b, const Move& m) {
    const bool w = b.white;
    if (m.null()) {
        b.ep = -1;
        ++b.halfmove;
        if (!w) ++b.fullmove;
        b.white = !w;
        return;
    }
    const int pc = b.sq[m.from], t = ptype(pc);
    const bool cap = is_capture(b, m);
    const bool ep_cap = is_ep_capture(b, m);
    const int ep_before = b.ep;
    b.ep = -1;
    b.halfmove = (cap || t == PAWN) ? 0 : b.halfmove + 1;
    if (!w) ++b.fullmove;
    // castling rights: any move from / to a corner or king square
    auto clear = [&](int s) {
        if (s == 0) b.castle &= ~CR_WQ;
        if (s == 7) b.castle &= ~CR_WK;
        if (s == 56) b.castle &= ~CR_BQ;
        if (s == 63) b.castle &= ~CR_BK;
        if (s == 4) b.castle &= ~(CR_WK | CR_WQ);
        if (s == 60) b.castle &= ~(CR_BK | CR_BQ);
    };
    clear(m.from);
    clear(m.to);
    if (t == KING) b.castle &= w ? ~(CR_WK | CR_WQ) : ~(CR_BK | CR_BQ);
    if (t == KING && abs(file_of(m.to) - file_of(m.from)) == 2) {
        const int r = rank_of(m.from);
        const bool ks = file_of(m.to) > file_of(m.from);
        const int rf = r * 8 + (ks ? 7 : 0), rt = r * 8 + (ks ? 5 : 3);
        b.sq[rt] = b.sq[rf];
        b.sq[rf] = 0;
    }
    if (ep_cap) b.sq[ep_before + (w ? -8 : 8)] = 0;
    b.sq[m.to] = m.promo ? mkpc(m.promo, w) : pc;
    b.sq[m.from] = 0;
    if (t == PAWN && abs(m.to - m.from) == 16) b.ep = (m.from + m.to) / 2;
    b.white = !w;
}

void gen_pseudo(const Board& b, std::vector<Move>& out) {
    const bool w = b.white;
    for (int s = 0; s < 64; ++s) {
        const int pc = b.sq[s];
        if (!pc || pwhite(pc) != w) continue;
        const int t = ptype(pc), f = file_of(s), r = rank_of(s);
        auto add = [&](int to) {
            if (t == PAWN && (rank_of(to) == 7 || rank_of(to) == 0)) {
                for (int p = QUEEN; p >= KNIGHT; --p) out.push_back({s, to, p});
            } else {
                out.push_back({s, to, 0});
            }
        };
        if (t == PAWN) {
            const int dr = w ? 1 : -1, start = w ? 1 : 6;
            if (on(f, r + dr) && !b.sq[(r + dr) * 8 + f]) {
                add((r + dr) * 8 + f);
                if (r == start && !b.sq[(r + 2 * dr) * 8 + f]) add((r + 2 * dr) * 8 + f);
            }
            for (int df = -1; df <= 1; df += 2) {
                if (!on(f + df, r + dr)) continue;
                const int to = (r + dr) * 8 + f + df;
                const int tp = b.sq[to];
                if ((tp && pwhite(tp) != w) || to == b.ep) add(to);
            }
        } else if (t == KNIGHT || t == KING) {
            const int(*D)[2] = t == KNIGHT ? KN_D : KG_D;
            for (int i = 0; i < 8; ++i) {
                const int ff = f + D[i][0], rr = r + D[i][1];
                if (!on(ff, rr)) continue;
                const int tp = b.sq[rr * 8 + ff];
                if (!tp || pwhite(tp) != w) add(rr * 8 + ff);
            }
        } else {
            for (int k = 0; k < 2; ++k) {
                if (k == 0 && t == BISHOP) continue;
                if (k == 1 && t == ROOK) continue;
                const int(*D)[2] = k == 0 ? RK_D : BS_D;
                for (int i = 0; i < 4; ++i) {
                    int ff = f + D[i][0], rr = r + D[i][1];
                    while (on(ff, rr)) {
                        const int tp = b.sq[rr * 8 + ff];
                        if (tp && pwhite(tp) == w) break;
                        add(rr * 8 + ff);
                        if (tp) break;
                        ff += D[i][0];
                        rr += D[i][1];
                    }
                }
            }
        }
    }
}

// legal castling moves (python-chess generate_castling_moves, standard chess)
void gen_castling(const Board& b, std::vector<Move>& out) {
    const bool w = b.white;
    const int base = w ? 0 : 56;
    if (b.sq[base + 4] != mkpc(KING, w) || attacked(b, base + 4, !w)) return;
    if ((b.castle & (w ? CR_WK : CR_BK)) && b.sq[base + 7] == mkpc(ROOK, w) && !b.sq[base + 5] && !b.sq[base + 6] &&
        !attacked(b, base + 5, !w) && !attacked(b, base + 6, !w))
        out.push_back({base + 4, base + 6, 0});
    if ((b.castle & (w ? CR_WQ : CR_BQ)) && b.sq[base + 0] == mkpc(ROOK, w) && !b.sq[base + 1] && !b.sq[base + 2] &&
        !b.sq[base + 3] && !attacked(b, base + 3, !w) && !attacked(b, base + 2, !w))
        out.push_back({base + 4, base + 2, 0});
}

bool legal_after(const Board& b, const Move& m) {
    Board c = b;
    push(c, m);
    const int k = king_sq(c, b.white);
    return k < 0 || !attacked(c, k, !b.white);
}

void gen_legal(const Board& b, std::vector<Move>& out) {
    std::vector<Move> ps;
    ps.reserve(64);
    gen_pseudo(b, ps);
    for (const Move& m : ps)
        if (legal_after(b, m)) out.push_back(m);
    gen_castling(b, out);
}

bool has_legal_ep(const Board& b) {
    if (b.ep < 0) return false;
    std::vector<Move> ms;
    gen_legal(b, ms);
    for (const Move& m : ms)
        if (is_ep_capture(b, m)) return true;
    return false;
}

std::string sq_name(int s) {
    std::string o;
    o += (char)('a' + file_of(s));
    o += (char)('1' + rank_of(s));
    return o;
}

// python-chess clean_castling_rights (standard): a right survives only with
// the king on its e-file square and the rook on its corner
int clean_castling(const Board& b) {
    int c = b.castle;
    if (b.sq[4] != mkpc(KING, true)) c &= ~(CR_WK | CR_WQ);
    if (b.sq[60] != mkpc(KING, false)) c &= ~(CR_BK | CR_BQ);
    if (b.sq[7] != mkpc(ROOK, true)) c &= ~CR_WK;
    if (b.sq[0] != mkpc(ROOK, true)) c &= ~CR_WQ;
    if (b.sq[63] != mkpc(ROOK, false)) c &= ~CR_BK;
    if (b.sq[56] != mkpc(ROOK, false)) c &= ~CR_BQ;
    return c;
}

std::string board_fen(const Board& b) {
    std::string o;
    for (int r = 7; r >= 0; --r) {
        int empty = 0;
        for (int f = 0; f < 8; ++f) {
            const int pc = b.sq[r * 8 + f];
            if (!pc) {
                ++empty;
                continue;
            }
            if (empty) o += (char)('0' + empty);
            empty = 0;
            o += PIECE_CHARS[pc];
        }
        if (empty) o += (char)('0' + empty);
        if (r) o += '/';
    }
    return o;
}

std::string fen(const Board& b) {
    std::string o = board_fen(b);
    o += b.white ? " w " : " b ";
    const int c = clean_castling(b);
    if (!c) o += '-';
    if (c & CR_WK) o += 'K';
    if (c & CR_WQ) o += 'Q';
    if (c & CR_BK) o += 'k';
    if (c & CR_BQ) o += 'q';
    o += ' ';
    o += has_legal_ep(b) ? sq_name(b.ep) : std::string("-");
    char tail[32];
    snprintf(tail, sizeof tail, " %d %d", b.halfmove, b.fullmove);
    return o + tail;
}

// python-chess Board.set_fen (standard chess); false on malformed text
bool set_fen(Board& b, const char* s) {
    Board n;
    memset(n.sq, 0, sizeof n.sq);
    std::vector<std::string> parts;
    std::string cur;
    for (const char* p = s; *p; ++p) {
        if (isspace((unsigned char)*p)) {
            if (!cur.empty()) parts.push_back(cur);
            cur.clear();
        } else {
            cur += *p;
        }
    }
    if (!cur.empty()) parts.push_back(cur);
    if (parts.empty() || parts.size() > 6) return false;
    int r = 7, f = 0;
    for (char ch : parts[0]) {
        if (ch == '/') {
            if (f != 8 || r == 0) return false;
            --r;
            f = 0;
        } else if (ch >= '1' && ch <= '8') {
            f += ch - '0';
            if (f > 8) return false;
        } else {
            const char* q = strchr(PIECE_CHARS + 1, ch);
            if (!q || f >= 8) return false;
            n.sq[r * 8 + f] = (int8_t)(q - PIECE_CHARS);
            ++f;
        }
    }
    if (r != 0 || f != 8) return false;
    if (parts.size() > 1) {
        if (parts[1] == "w") n.white = true;
        else if (parts[1] == "b") n.white = false;
        else return false;
    }
    if (parts.size() > 2 && parts[2] != "-") {
        for (char ch : parts[2]) {
            if (ch == 'K') n.castle |= CR_WK;
            else if (ch == 'Q') n.castle |= CR_WQ;
            else if (ch == 'k') n.castle |= CR_BK;
            else if (ch == 'q') n.castle |= CR_BQ;
            else return false;
        }
    }
    if (parts.size() > 3 && parts[3] != "-") {
        const std::string& e = parts[3];
        if (e.size() != 2 || e[0] < 'a' || e[0] > 'h' || e[1] < '1' || e[1] > '8') return false;
        n.ep = (e[1] - '1') * 8 + (e[0] - 'a');
    }
    if (parts.size() > 4) n.halfmove = atoi(parts[4].c_str());
    if (parts.size() > 5) n.fullmove = atoi(parts[5].c_str());
    if (n.fullmove < 1) n.fullmove = 1;
    b = n;
    return true;
}

void starting(Board& b) { set_fen(b, "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"); }

std::string san(const Board& b, const Move& m) {
    if (m.null()) return "--";
    std::string o;
    if (is_castling(b, m)) {
        o = file_of(m.to) < file_of(m.from) ? "O-O-O" : "O-O";
    } else {
        const int t = ptype(b.sq[m.from]);
        const bool cap = is_capture(b, m);
        if (t != PAWN) {
            o += PIECE_CHARS[t];
            std::vector<Move> ms;
            gen_legal(b, ms);
            uint64_t others = 0;
            for (const Move& c : ms)
                if (c.to == m.to && c.from != m.from && ptype(b.sq[c.from]) == t) others |= 1ull << c.from;
            if (others) {
                bool row = false, column = false;
                const uint64_t rank_mask = 0xFFull << (8 * rank_of(m.from));
                const uint64_t file_mask = 0x0101010101010101ull << file_of(m.from);
                if (others & rank_mask) column = true;
                if (others & file_mask) row = true;
                else column = true;
                if (column) o += (char)('a' + file_of(m.from));
                if (row) o += (char)('1' + rank_of(m.from));
            }
        } else if (cap) {
            o += (char)('a' + file_of(m.from));
        }
        if (cap) o += 'x';
        o += sq_name(m.to);
        if (m.promo) {
            o += '=';
            o += PIECE_CHARS[m.promo];
        }
    }
    Board c = b;
    push(c, m);
    if (in_check(c)) {
        std::vector<Move> ms;
        gen_legal(c, ms);
        o += ms.empty() ? '#' : '+';
    }
    return o;
}

// python-chess Board.parse_san; returns 0 and the move, or -1 with *err set
int parse_san(const Board& b, const std::string& s, Move& out, std::string& err) {
    static const char* KS[] = {"O-O", "O-O+", "O-O#", "0-0", "0-0+", "0-0#"};
    static const char* QS[] = {"O-O-O", "O-O-O+", "O-O-O#", "0-0-0", "0-0-0+", "0-0-0#"};
    for (int k = 0; k < 2; ++k) {
        const char** L = k == 0 ? KS : QS;
        for (int i = 0; i < 6; ++i) {
            if (s != L[i]) continue;
            std::vector<Move> cs;
            gen_castling(b, cs);
            for (const Move& m : cs)
                if ((file_of(m.to) > file_of(m.from)) == (k == 0)) {
                    out = m;
                    return 0;
                }
            err = "illegal san: '" + s + "' in " + fen(b);
            return -1;
        }
    }
    // ^([NBKRQ])?([a-h])?([1-8])?[\-x]?([a-h][1-8])(=?[nbrqkNBRQK])?[\+#]?\Z
    size_t i = 0;
    const size_t n = s.size();
    int piece = 0, ffile = -1, frank = -1, to = -1, promo = 0;
    bool ok = true;
    auto fail = [&]() { ok = false; };
    if (i < n && strchr("NBKRQ", s[i]) && s[i]) {
        piece = (int)(strchr(PIECE_CHARS, s[i]) - PIECE_CHARS);
        ++i;
    }
    // the regex is greedy with backtracking: a bare "[a-h][1-8]" is the target square. Collect the optional
    // from-file / from-rank only when a target square still follows.
    auto is_file = [&](size_t k) { return k < n && s[k] >= 'a' && s[k] <= 'h'; };
    auto is_rank = [&](size_t k) { return k < n && s[k] >= '1' && s[k] <= '8'; };
    auto tail_ok = [&](size_t k) {  // ([a-h][1-8])(=?[nbrqkNBRQK])?[\+#]?$ from k (after an optional [-x])
        if (k < n && (s[k] == '-' || s[k] == 'x')) ++k;
        if (!(is_file(k) && is_rank(k + 1))) return false;
        k += 2;
        if (k < n && s[k] == '=') ++k;
        if (k < n && strchr("nbrqkNBRQK", s[k]) && s[k]) ++k;
        else if (k > 0 && s[k - 1] == '=') return false;
        if (k < n && (s[k] == '+' || s[k] == '#')) ++k;
        return k == n;
    };
    if (is_file(i) && is_rank(i + 1) && tail_ok(i + 2)) {
        ffile = s[i] - 'a';
        frank = s[i + 1] - '1';
        i += 2;
    } else if (is_file(i) && tail_ok(i + 1)) {
        ffile = s[i] - 'a';
        i += 1;
    } else if (is_rank(i) && tail_ok(i + 1)) {
        frank = s[i] - '1';
        i += 1;
    }
    if (!tail_ok(i)) fail();
    if (ok) {
        if (s[i] == '-' || s[i] == 'x') ++i;
        to = (s[i + 1] - '1') * 8 + (s[i] - 'a');
        i += 2;
        if (i < n && s[i] == '=') ++i;
        if (i < n && strchr("nbrqkNBRQK", s[i]) && s[i]) {
            promo = (int)(strchr(PIECE_CHARS, toupper((unsigned char)s[i])) - PIECE_CHARS);
            ++i;
        }
    }
    if (!ok) {
        if (s == "--" || s == "Z0" || s == "0000" || s == "@@@@") {
            out = Move{0, 0, 0};
            return 0;
        }
        err = (s.find(',') != std::string::npos ? "unsupported multi-leg move: '" : "invalid san: '") + s + "'";
        return -1;
    }
    std::vector<Move> ms;
    gen_legal(b, ms);
    if (!piece && ffile >= 0 && frank >= 0) {
        // fully specified from-square (python-chess find_move): any legal move from there, castling included;
        // king-takes-own-rook spellings e1h1 / e1a1 (e8h8 / e8a8) mean castling (_from_chess960)
        const int from = frank * 8 + ffile;
        if (!promo && ptype(b.sq[from]) == KING && (from == 4 || from == 60) && rank_of(to) == rank_of(from)) {
            if (file_of(to) == 7) to = from + 2;
            else if (file_of(to) == 0) to = from - 2;
        }
        const Move* found = nullptr;
        for (const Move& m : ms)
            if (m.from == from && m.to == to && (m.promo == promo || (!promo && m.promo == QUEEN))) {
                // find_move defaults a missing promotion to a queen, then parse_san requires it to match
                if (m.promo == promo || !found) found = &m;
            }
        if (!found) {
            err = "illegal san: '" + s + "' in " + fen(b);
            return -1;
        }
        if (found->promo != promo) {
            err = "missing promotion piece type: '" + s + "' in " + fen(b);
            return -1;
        }
        out = *found;
        return 0;
    }
    // "Mask our own pieces to exclude castling moves"
    if (b.sq[to] && pwhite(b.sq[to]) == b.white) {
        err = "illegal san: '" + s + "' in " + fen(b);
        return -1;
    }
    const Move* match = nullptr;
    for (const Move& m : ms) {
        if (m.to != to || m.promo != promo) continue;
        const int t = ptype(b.sq[m.from]);
        if (piece ? t != piece : t != PAWN) continue;
        if (ffile >= 0 && file_of(m.from) != ffile) continue;
        if (frank >= 0 && rank_of(m.from) != frank) continue;
        if (!piece && ffile < 0 && file_of(m.from) != file_of(to)) continue;  // no pawn capture without a file
        if (match) {
            err = "ambiguous san: '" + s + "' in " + fen(b);
            return -1;
        }
        match = &m;
    }
    if (!match) {
        err = "illegal san: '" + s + "' in " + fen(b);
        return -1;
    }
    out = *match;
    return 0;
}

uint64_t perft(const Board& b, int depth) {
    std::vector<Move> ms;
    gen_legal(b, ms);
    if (depth == 1) return ms.size();
    uint64_t n = 0;
    for (const Move& m : ms) {
        Board c = b;
        push(c, m);
        n += perft(c, depth - 1);
    }
    return n;
}

// ------------------------------------------------------------------ PGN --
struct PgnGame {
    Board start;
    std::string result = "*";
    std::vector<Move> moves;  // mainline up to the first error
    bool bad_fen = false;
};

struct PgnReader {
    const char* p;
    const char* end;
    PgnReader(const char* t, size_t n) : p(t), end(t + n) {}
    bool eof() const { return p >= end; }
    // one line including its newline; empty string at EOF
    std::string readline() {
        const char* s = p;
        while (p < end && *p != '\n') ++p;
        if (p < end) ++p;
        return std::string(s, p);
    }
};

bool is_space_line(const std::string& l) {
    if (l.empty()) return false;  // EOF marker
    for (char c : l)
        if (!isspace((unsigned char)c)) return false;
    return true;
}

bool starts(const std::string& l, char c) { return !l.empty() && l[0] == c; }

// TAG_REGEX ^\[([A-Za-z0-9][A-Za-z0-9_+#=:-]*)\s+\"([^\r]*)\"\]\s*$
bool parse_tag(const std::string& line, std::string& key, std::string& val) {
    size_t i = 1, n = line.size();
    if (i >= n || !isalnum((unsigned char)line[i])) return false;
    size_t k0 = i;
    while (i < n && (isalnum((unsigned char)line[i]) || strchr("_+#=:-", line[i]))) ++i;
    key = line.substr(k0, i - k0);
    if (i >= n || !isspace((unsigned char)line[i])) return false;
    while (i < n && isspace((unsigned char)line[i])) ++i;
    if (i >= n || line[i] != '"') return false;
    // value: greedy up to the last '"' followed by ']' and trailing whitespace
    size_t j = n;
    while (j > i && isspace((unsigned char)line[j - 1])) --j;
    if (j < i + 2 || line[j - 1] != ']' || line[j - 2] != '"') return false;
    val = line.substr(i + 1, j - 2 - (i + 1));
    if (val.find('\r') != std::string::npos) return false;
    return true;
}

// chess.pgn.read_game semantics for the mainline; returns false at end of input
bool read_game(PgnReader& rd, PgnGame& g) {
    g = PgnGame();
    starting(g.start);
    std::string line = rd.readline();
    if (line.size() >= 3 && (unsigned char)line[0] == 0xEF && (unsigned char)line[1] == 0xBB &&
        (unsigned char)line[2] == 0xBF)
        line = line.substr(3);
    while (is_space_line(line) || starts(line, '%') || starts(line, ';')) line = rd.readline();
    bool found = false;
    int consecutive_empty = 0;
    std::string fen_tag;
    bool have_fen = false;
    while (!line.empty()) {
        if (starts(line, '%') || starts(line, ';')) {
            line = rd.readline();
            continue;
        }
        if (consecutive_empty < 1 && is_space_line(line)) {
            ++consecutive_empty;
            line = rd.readline();
            continue;
        }
        found = true;
        if (!starts(line, '[')) break;
        consecutive_empty = 0;
        std::string k, v;
        if (parse_tag(line, k, v)) {
            if (k == "Result") g.result = v;
            if (k == "FEN") {
                fen_tag = v;
                have_fen = true;
            }
        }
        line = rd.readline();
    }
    if (!found) return false;
    if (have_fen) {
        Board fb;
        if (!set_fen(fb, fen_tag.c_str())) g.bad_fen = true;
        else g.start = fb;
    }
    while (is_space_line(line)) line = rd.readline();
    Board board = g.start;
    int depth = 0;          // variation nesting below the mainline
    bool skip_main = g.bad_fen;  // after a mainline error: the rest of the mainline is skipped
    while (!line.empty()) {
        if (starts(line, '%') || starts(line, ';')) {
            line = rd.readline();
            continue;
        }
        if (is_space_line(line)) return true;  // an empty line ends the game
        size_t i = 0;
        size_t n = line.size();
        while (i < n) {
            const char c = line[i];
            if (c == '{') {  // comment, possibly spanning lines
                size_t j = line.find('}', i + 1);
                while (j == std::string::npos) {
                    line = rd.readline();
                    if (line.empty()) return true;
                    n = line.size();
                    j = line.find('}');
                }
                i = j + 1;
                continue;
            }
            if (c == ';') break;  // comment to end of line
            if (c == '(') {
                ++depth;
                ++i;
                continue;
            }
            if (c == ')') {
                if (depth) --depth;
                ++i;
                continue;
            }
            if (c == '$') {
                ++i;
                while (i < n && isdigit((unsigned char)line[i])) ++i;
                continue;
            }
            // results
            if (line.compare(i, 7, "1/2-1/2") == 0) {
                if (!depth && g.result == "*") g.result = "1/2-1/2";
                i += 7;
                continue;
            }
            if (line.compare(i, 3, "1-0") == 0 || line.compare(i, 3, "0-1") == 0) {
                // "0-1" vs castling "0-0": distinct texts
                if (!depth && g.result == "*") g.result = line.substr(i, 3);
                i += 3;
                continue;
            }
            if (c == '*') {
                if (!depth && g.result == "*") g.result = "*";
                ++i;
                continue;
            }
            // move tokens (MOVETEXT_REGEX alternatives, longest first)
            size_t j = i;
            std::string tok;
            auto take = [&](const char* lit) {
                const size_t L = strlen(lit);
                if (line.compare(i, L, lit) == 0) {
                    tok = lit;
                    j = i + L;
                    return true;
                }
                return false;
            };
            if (take("O-O-O") || take("O-O") || take("0-0-0") || take("0-0") || take("--") || take("Z0") ||
                take("0000") || take("@@@@")) {
            } else {
                // [NBKRQ]?[a-h]?[1-8]?[\-x]?[a-h][1-8](?:=?[nbrqkNBRQK])?  |  [PNBRQK]?@[a-h][1-8]
                size_t k = i;
                bool drop = false;
                if (k < n && strchr("PNBRQK", line[k]) && line[k] && k + 1 < n && line[k + 1] == '@') {
                    drop = true;
                    k += 2;
                } else if (k < n && line[k] == '@') {
                    drop = true;
                    k += 1;
                }
                if (drop) {
                    if (k + 1 < n && line[k] >= 'a' && line[k] <= 'h' && line[k + 1] >= '1' && line[k + 1] <= '8') {
                        tok = line.substr(i, k + 2 - i);
                        j = k + 2;
                    }
                } else {
                    // try the SAN shape with the regex's backtracking: longest match that ends on a square
                    size_t best = 0;
                    for (size_t len = 1; len <= 9 && i + len <= n; ++len) {
                        std::string cand = line.substr(i, len);
                        // validate cand against ^[NBKRQ]?[a-h]?[1-8]?[-x]?[a-h][1-8](=?[nbrqkNBRQK])?$
                        size_t q = 0, m = cand.size();
                        if (q < m && strchr("NBKRQ", cand[q]) && cand[q]) ++q;
                        bool okc = false;
                        for (int opt = 0; opt < 8 && !okc; ++opt) {
                            size_t r2 = q;
                            if ((opt & 1) && r2 < m && cand[r2] >= 'a' && cand[r2] <= 'h') ++r2;
                            else if (opt & 1) continue;
                            if ((opt & 2) && r2 < m && cand[r2] >= '1' && cand[r2] <= '8') ++r2;
                            else if (opt & 2) continue;
                            if ((opt & 4) && r2 < m && (cand[r2] == '-' || cand[r2] == 'x')) ++r2;
                            else if (opt & 4) continue;
                            if (!(r2 + 1 < m + 1 && r2 + 2 <= m && cand[r2] >= 'a' && cand[r2] <= 'h' &&
                                  cand[r2 + 1] >= '1' && cand[r2 + 1] <= '8'))
                                continue;
                            r2 += 2;
                            if (r2 == m) okc = true;
                            else if (r2 + 1 == m && strchr("nbrqkNBRQK", cand[r2]) && cand[r2]) okc = true;
                            else if (r2 + 2 == m && cand[r2] == '=' && strchr("nbrqkNBRQK", cand[r2 + 1]) &&
                                     cand[r2 + 1])
                                okc = true;
                        }
                        if (okc) best = len;
                    }
                    if (best) {
                        tok = line.substr(i, best);
                        j = i + best;
                    }
                }
            }
            if (tok.empty()) {  // not a token: skip one character (move numbers, '+', '#', '.', glyphs, ...)
                ++i;
                continue;
            }
            i = j;
            if (depth || skip_main) continue;
            Move m;
            std::string err;
            if (tok.find('@') != std::string::npos || parse_san(board, tok, m, err) != 0) {
                skip_main = true;  // GameBuilder.handle_error + skip the rest of the mainline
                continue;
            }
            g.moves.push_back(m);
            push(board, m);
        }
        line = rd.readline();
    }
    return true;
}

int outcome_of(const std::string& r) {
    if (r == "1-0") return 1;
    if (r == "0-1") return -1;
    if (r == "1/2-1/2") return 0;
    return KV_PGN_OUTCOME_NONE;
}

void copy_str(char* dst, size_t cap, const std::string& s) {
    const size_t n = s.size() < cap - 1 ? s.size() : cap - 1;
    memcpy(dst, s.data(), n);
    memset(dst + n, 0, cap - n);
}

}  // namespace

extern "C" {

int kv_pgn_extract(const char* text, size_t len, kv_pgn_record* out, size_t cap, size_t* n_out, size_t* consumed,
                   int64_t* n_games) {
    if (!text || !n_out || !consumed || !n_games) {
        kv::set_error("kv_pgn_extract: NULL argument");
        return KV_EINVAL;
    }
    PgnReader rd(text, len);
    size_t n = 0;
    int64_t games = 0;
    *consumed = 0;
    PgnGame g;
    while (true) {
        const char* game_start = rd.p;
        if (!read_game(rd, g)) {
            *consumed = len;
            break;
        }
        if (n + g.moves.size() > cap) {
            if (n == 0) {
                kv::set_error("kv_pgn_extract: one game has %zu moves, buffer holds %zu", g.moves.size(), cap);
                *n_out = g.moves.size();
                return KV_EOVERFLOW;
            }
            rd.p = game_start;  // the next call starts here
            break;
        }
        Board b = g.start;
        const int oc = outcome_of(g.result);
        for (const Move& m : g.moves) {
            kv_pgn_record& r = out[n++];
            copy_str(r.fen, sizeof r.fen, fen(b));
            copy_str(r.san, sizeof r.san, san(b, m));
            r.outcome = oc;
            r.game = (int32_t)games;
            push(b, m);
        }
        ++games;
        *consumed = (size_t)(rd.p - text);
    }
    *n_out = n;
    *n_games = games;
    return KV_OK;
}

int kv_fen_codes(const char* fens, size_t stride, int n, int8_t* codes) {
    if ((!fens || !codes) && n > 0) {
        kv::set_error("kv_fen_codes: NULL argument");
        return KV_EINVAL;
    }
    for (int i = 0; i < n; ++i) {
        Board b;
        if (!set_fen(b, fens + (size_t)i * stride)) {
            kv::set_error("kv_fen_codes: invalid fen at row %d: '%.90s'", i, fens + (size_t)i * stride);
            return KV_EINVAL;
        }
        // PGN plane order P N B R Q K p n b r q k (codes 1..12), row 0 = rank 8 (dataset.py:63-67)
        for (int s = 0; s < 64; ++s) codes[(size_t)i * 64 + (7 - rank_of(s)) * 8 + file_of(s)] = b.sq[s];
    }
    return KV_OK;
}

int kv_san_move_index(const char* fens, size_t fen_stride, const char* sans, size_t san_stride, int n,
                      int32_t* out) {
    if ((!fens || !sans || !out) && n > 0) {
        kv::set_error("kv_san_move_index: NULL argument");
        return KV_EINVAL;
    }
    for (int i = 0; i < n; ++i) {
        Board b;
        if (!set_fen(b, fens + (size_t)i * fen_stride)) {
            kv::set_error("kv_san_move_index: invalid fen at row %d", i);
            return KV_EINVAL;
        }
        Move m;
        std::string err;
        if (parse_san(b, std::string(sans + (size_t)i * san_stride), m, err) != 0) {
            kv::set_error("kv_san_move_index: row %d: %s", i, err.c_str());
            return KV_EINVAL;
        }
        out[i] = m.from * 64 + m.to;  // scripts/train.py:553-558 (python-chess squares; null move -> 0)
    }
    return KV_OK;
}

int kv_chess_perft(const char* fen_text, int depth, uint64_t* nodes) {
    Board b;
    if (!fen_text || !nodes || depth < 1 || !set_fen(b, fen_text)) {
        kv::set_error("kv_chess_perft: bad argument");
        return KV_EINVAL;
    }
    *nodes = perft(b, depth);
    return KV_OK;
}

int kv_chess_san(const char* fen_text, const char* san_in, char* san_out, size_t san_cap, char* fen_after,
                 size_t fen_cap) {
    Board b;
    if (!fen_text || !san_in || !san_out || san_cap < 2 || !set_fen(b, fen_text)) {
        kv::set_error("kv_chess_san: bad argument");
        return KV_EINVAL;
    }
    Move m;
    std::string err;
    if (parse_san(b, san_in, m, err) != 0) {
        kv::set_error("%s", err.c_str());
        return KV_EINVAL;
    }
    copy_str(san_out, san_cap, san(b, m));
    push(b, m);
    if (fen_after && fen_cap > 1) copy_str(fen_after, fen_cap, fen(b));
    return KV_OK;
}

int kv_chess_fen(const char* fen_in, char* fen_out, size_t cap) {
    Board b;
    if (!fen_in || !fen_out || cap < 2 || !set_fen(b, fen_in)) {
        kv::set_error("kv_chess_fen: invalid fen '%.90s'", fen_in ? fen_in : "(null)");
        return KV_EINVAL;
    }
    copy_str(fen_out, cap, fen(b));
    return KV_OK;
}

}  // extern "C"
