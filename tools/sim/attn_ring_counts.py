"""Design check for k_attn_bf16_ring's counted vmcnt waits (csrc/attention.hip): simulate one wave's vector-memory
issue sequence and verify that the closed-form wait counts the kernel uses equal the number of ops issued after the
newest op each wait needs (so, with in-order retirement, the wait retires exactly that op and everything older), for
every (NT, R, CB, J, S) combination.

Per wave, in issue order:
  prologue: Q(0) pieces x4 (the wave's query strip of unit 0 -> its LDS Q area), chunk pieces 0 .. R-CB-1;
  for every unit j, for every chunk c (g = j NT + c):
    group top (g % CB == 0): wait for the piece of chunk g + CB - 1 [k_gt], barrier, pieces g+R-CB .. g+R-1;
    unit start (c == 0): wait for the Q(j) pieces [k_qw], read Q(j) from LDS, then Q(j+1) pieces x4;
    compute chunk g;
  unit end: S output stores."""
import itertools


def k_gt(s, NT, R, CB, S):
    """Ops issued after the piece of chunk gl = s CB + CB - 1, seen at group top s."""
    gl = s * CB + CB - 1
    si = max(0, (gl - R + CB) // CB)      # group whose top issued piece gl (prologue -> 0)
    a, b = si * CB, s * CB
    nq = (b - 1) // NT - (a - 1) // NT if b > a else 0          # unit starts j NT in [a, b)  (j >= 0)
    ns = b // NT - a // NT                                       # unit ends m NT in (a, b]  (m >= 1)
    return (R - 2 * CB) + 4 * nq + S * ns


def k_qw(j, NT, R, CB, S):
    """Ops issued after the last Q(j) piece, seen at unit j's start (after the group top of chunk j NT, if any)."""
    if j == 0:
        return R   # Q(0) is the oldest op: the R - CB prologue pieces and group top 0's CB pieces follow it
    gts = (j * NT) // CB - ((j - 1) * NT) // CB                  # group tops in ((j-1) NT, j NT]
    return CB * gts + S


def simulate(NT, R, CB, J, S):
    G = J * NT
    seq = [("Q", 0)] * 4 + [("P", g) for g in range(R - CB)]

    def after(tag):
        return len(seq) - 1 - max(i for i, t in enumerate(seq) if t == tag)
    for j in range(J):
        for c in range(NT):
            g = j * NT + c
            if g % CB == 0:
                s = g // CB
                assert after(("P", s * CB + CB - 1)) == k_gt(s, NT, R, CB, S), ("gt", NT, R, CB, J, S, s)
                seq += [("P", x) for x in range(s * CB + R - CB, s * CB + R)]
            if c == 0:
                assert after(("Q", j)) == k_qw(j, NT, R, CB, S), ("qw", NT, R, CB, J, S, j)
                seq += [("Q", j + 1)] * 4
        seq += [("S", j)] * S
    return True


if __name__ == "__main__":
    n = 0
    for NT, R, CB, J, S in itertools.product(range(1, 9), range(2, 11), range(1, 6), range(1, 6), (0, 4, 5)):
        if R < 2 * CB:
            continue
        simulate(NT, R, CB, J, S)
        n += 1
    print(f"ok: {n} configurations")
