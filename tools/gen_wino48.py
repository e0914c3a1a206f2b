"""Exact Toom-Cook matrices of Winograd F(8,3) (the 8-wide axis of the
F(4x8, 3x3) tower, csrc/kv_wino48.h): points 0, +-1, +-1/2, +-2, +-3/4, inf.
A^T[i][j] = p_j^i, G[j][k] = p_j^k / prod_{l != j}(p_j - p_l), B^T solved
exactly so that A^T ((G g) * (B^T d)) is the 8-output correlation of d (10)
with g (3). Prints the C tables; every A^T / B^T entry is a dyadic rational
(exact in fp32), G is applied in fp64 and rounded once.

    python tools/gen_wino48.py
"""
from fractions import Fraction as Fr
import itertools

P = [Fr(0), Fr(1), Fr(-1), Fr(1, 2), Fr(-1, 2), Fr(2), Fr(-2), Fr(3, 4), Fr(-3, 4)]
M, R = 8, 3
N = M + R - 1


def matrices():
    AT = [[Fr(0)] * N for _ in range(M)]
    G = [[Fr(0)] * R for _ in range(N)]
    for j, a in enumerate(P):
        den = Fr(1)
        for l, b in enumerate(P):
            if l != j:
                den *= a - b
        for i in range(M):
            AT[i][j] = a ** i
        for k in range(R):
            G[j][k] = a ** k / den
    AT[M - 1][N - 1] = Fr(1)
    G[N - 1][R - 1] = Fr(1)
    # B^T rows from the Lagrange structure: solve the linear system exactly (Gauss-Jordan over Fractions)
    unknowns = N * N
    rows, rhs = [], []
    for i in range(M):
        for k in range(R):
            for l in range(N):
                row = [Fr(0)] * unknowns
                for j in range(N):
                    row[j * N + l] = AT[i][j] * G[j][k]
                rows.append(row)
                rhs.append(Fr(1) if l == i + k else Fr(0))
    # least-norm exact solution of a consistent system: eliminate, free variables = 0
    A = [r[:] + [b] for r, b in zip(rows, rhs)]
    piv_cols, r = [], 0
    for c in range(unknowns):
        p = next((q for q in range(r, len(A)) if A[q][c] != 0), None)
        if p is None:
            continue
        A[r], A[p] = A[p], A[r]
        inv = 1 / A[r][c]
        A[r] = [x * inv for x in A[r]]
        for q in range(len(A)):
            if q != r and A[q][c] != 0:
                f = A[q][c]
                A[q] = [x - f * y for x, y in zip(A[q], A[r])]
        piv_cols.append(c)
        r += 1
    assert all(all(x == 0 for x in row[:-1]) <= (row[-1] == 0) for row in A[r:]), "inconsistent"
    sol = [Fr(0)] * unknowns
    for q, c in enumerate(piv_cols):
        sol[c] = A[q][-1]
    BT = [[sol[j * N + l] for l in range(N)] for j in range(N)]
    # verify on the basis
    for i, k, l in itertools.product(range(M), range(R), range(N)):
        s = sum(AT[i][j] * G[j][k] * BT[j][l] for j in range(N))
        assert s == (1 if l == i + k else 0)
    return AT, G, BT


def dyadic(x):
    d = x.denominator
    return d & (d - 1) == 0


def ctab(name, T, ctype="float"):
    out = [f"__constant__ const {ctype} {name}[{len(T)}][{len(T[0])}] = {{"]
    for row in T:
        out.append("    {" + ", ".join(repr(float(x)) for x in row) + "},")
    out.append("};")
    return "\n".join(out)


if __name__ == "__main__":
    AT, G, BT = matrices()
    assert all(dyadic(x) for row in AT + BT for x in row)
    print(ctab("kW8_AT", AT))
    print(ctab("kW8_BT", BT))
    print(ctab("kW8_G", G, "double"))


def fma_chain(T, n_in, name, n_out):
    """C body: o[r] = sum_j T[r][j] * d[j], as an explicit fmaf chain in j order
    (zeros skipped, first term a plain product / copy) -- the same bits at every
    call site, whatever the compiler's contraction choices."""
    lines = [f"__device__ inline void {name}(const float* d, float* o) {{"]
    for r in range(n_out):
        terms = [(j, T[r][j]) for j in range(n_in) if T[r][j] != 0]
        expr = None
        for j, c in terms:
            cf = repr(float(c)) + "f"
            if expr is None:
                expr = f"d[{j}]" if c == 1 else (f"-d[{j}]" if c == -1 else f"{cf} * d[{j}]")
            else:
                expr = f"__builtin_fmaf({cf}, d[{j}], {expr})"
        lines.append(f"    o[{r}] = {expr};")
    lines.append("}")
    return "\n".join(lines)


def emit_device():
    AT, G, BT = matrices()
    return "\n\n".join([fma_chain(BT, N, "w8_bt", N), fma_chain(AT, N, "w8_at", M)])
