"""The batched per-party tail (csrc/rss_jobs.hip, ring.jobs_r0/r1/r2): several products
of one round in the tail's three kernels, each job's cross terms computed inside round 0
and its new shares written straight to its output rows, are bitwise the shares of the
generic path -- every pair's cross terms, concatenated, then the per-party dot tail
(k_dot_tail_r0/r1/r2) and the slices of its output (fixedpoint._merged_exp_tail's rounds)."""
import pytest
import torch

from moose_amd.ops import ring as R
from moose_amd.runtime.keys import KeyTable


def _rand(shape, bits, g, device):
    t = torch.randint(-(1 << 62), 1 << 62, tuple(shape) + ((2,) if bits == 128 else ()),
                      generator=g, dtype=torch.int64)
    return t.to(device)


def _shares(rows, L, bits, g, device):
    """Replicated shares of a random [rows, L] value: party p holds (x_p, x_{p+1})."""
    x = [_rand((rows, L), bits, g, device) for _ in range(3)]
    return [(x[p], x[(p + 1) % 3]) for p in range(3)]


def _run_rounds(r0, r1, r2):
    """Route the messages of the three parties through rounds A and B of the dot tail."""
    msg, rt, rm = zip(*[r0(p) for p in range(3)])
    # round A: m0 -> P1, m1 -> P0, z2 -> P0 and P1, rt1 / rm1 -> P1
    rmk = [msg[1], msg[0], None]
    w = [r1(p, msg[p], rmk[p], msg[2], rt[2] if p == 1 else None, rm[2] if p == 1 else None)
         for p in range(3)]
    # round B: w0 <-> w1
    r2(0, w[0], w[1])
    r2(1, w[1], w[0])


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("bits", [64, 128])
def test_jobs_tail_bitwise_equals_cross_concat_tail(device, bits):
    g = torch.Generator().manual_seed(bits)
    kt = KeyTable(device, capacity=8)
    base = kt.alloc(3)
    slots = [[kt.ptr(base + p), kt.ptr(base + (p + 1) % 3)] for p in range(3)]
    L, m = 6, 37
    nonces = tuple(range(101, 108))
    # a polynomial level: x^h (one row, broadcast) times P[0:2]; a tree level: F[0:2] * F[2:4];
    # 3 a - 5 b for additive shares a, b (first share components), all in one round
    xh = _shares(1, L, bits, g, device)
    P = _shares(2, L, bits, g, device)
    F = _shares(4, L, bits, g, device)
    A = _shares(1, L, bits, g, device)
    B = _shares(1, L, bits, g, device)
    rows = 2 + 2 + 1

    # --- generic: cross terms per pair, concatenated, then the dot tail on the whole
    def cross(x0, x1, y0, y1):
        return R.rss_cross("arith", R.RT(x0, bits), R.RT(x1, bits), R.RT(y0, bits),
                           R.RT(y1, bits), None, 0, 1).data

    def generic_parts(p):
        a = cross(xh[p][0].expand(2, L, *xh[p][0].shape[2:]).contiguous(),
                  xh[p][1].expand(2, L, *xh[p][1].shape[2:]).contiguous(), P[p][0], P[p][1])
        b = cross(F[p][0][0:2], F[p][1][0:2], F[p][0][2:4], F[p][1][2:4])
        k = lambda v: R.fill((), v % (1 << bits), bits, device)  # noqa: E731
        c = R.binary("add", R.binary("mul", R.RT(A[p][0], bits), k(3)),
                     R.binary("mul", R.RT(B[p][0], bits), k(-5))).data
        return torch.cat([a, b, c], 0).contiguous()

    gen_out = [(torch.empty_like(generic_parts(p)), torch.empty_like(generic_parts(p)))
               for p in range(3)]
    n_el = rows * L

    def g_r0(p):
        c = generic_parts(p)
        msg, rt, rm = R.dot_tail_r0([c], bits, m, [p], slots[p], nonces, [gen_out[p][0]],
                                    [gen_out[p][1]], n_el)
        return msg[0], rt[0], rm[0]

    def g_r1(p, msg, rmk, z2, rrt, rrm):
        if p == 2:
            return None
        return R.dot_tail_r1([msg], [rmk], [z2], [rrt], [rrm], bits, m, [p], slots[p], nonces,
                             [gen_out[p][0]], [gen_out[p][1]], n_el)[0]

    def g_r2(p, a, b):
        R.dot_tail_r2([a], [b], [gen_out[p][1] if p == 0 else gen_out[p][0]], bits, [p], n_el)

    _run_rounds(g_r0, g_r1, g_r2)

    # --- jobs: the same three products written to separate output buffers
    outs = [[(torch.empty_like(P[p][0]), torch.empty_like(P[p][0])),
             (torch.empty_like(F[p][0][0:2]), torch.empty_like(F[p][0][0:2])),
             (torch.empty_like(A[p][0]), torch.empty_like(A[p][0]))] for p in range(3)]

    def jobs(p):
        (o0a, o1a), (o0b, o1b), (o0c, o1c) = outs[p]
        return [R.MulJob(2, o0a, o1a, x=xh[p], y=P[p], sx=0, sy=L),
                R.MulJob(2, o0b, o1b, x=(F[p][0][0:2], F[p][1][0:2]),
                         y=(F[p][0][2:4], F[p][1][2:4]), sx=L, sy=L),
                R.MulJob(1, o0c, o1c, a=A[p][0], sa=L, ca=3, a2=B[p][0], sa2=L, ca2=-5)]

    def j_r0(p):
        return R.jobs_r0(jobs(p), L, bits, m, p, slots[p], nonces, like=P[p][0])

    def j_r1(p, msg, rmk, z2, rrt, rrm):
        return R.jobs_r1(jobs(p), L, bits, m, p, slots[p], nonces, msg, rmk, z2, rrt, rrm)

    def j_r2(p, a, b):
        R.jobs_r2(jobs(p), L, bits, p, a, b)

    _run_rounds(j_r0, j_r1, j_r2)
    for p in range(3):
        want0, want1 = gen_out[p]
        got0 = torch.cat([o[0] for o in outs[p]], 0)
        got1 = torch.cat([o[1] for o in outs[p]], 0)
        assert torch.equal(got0.reshape(want0.shape).cpu(), want0.cpu()), p
        assert torch.equal(got1.reshape(want1.shape).cpu(), want1.cpu()), p
