"""Design check for k_attn_bf16_ring's counted vmcnt waits (csrc/attention.hip): simulate one wave's vector-memory
issue sequence (Q loads, one K/V DMA piece per chunk, output stores) and verify that the closed-form wait count the
kernel uses at every group top equals the number of ops issued after the newest piece it needs (so the wait retires
exactly that piece and everything older, with in-order retirement), for every (NT, R, CB, J, S) combination used."""
import itertools


def ring_wait_count(s, NT, R, CB, S):
    """The kernel's formula: ops issued after the piece of chunk s*CB + CB - 1, seen at group top s. Unit boundaries
    (the next unit's 4 Q loads + this unit's S stores) are issued after a unit's last chunk is computed, i.e. after
    chunk m*NT - 1 for m = 1, 2, ...: those computed in groups s_issue .. s - 1 come after piece gl."""
    gl = s * CB + CB - 1
    s_issue = max(0, (gl - R + CB) // CB)          # group whose top issued piece gl (prologue -> 0)
    bound = (s * CB) // NT - (s_issue * CB) // NT
    return (R - 2 * CB) + (4 + S) * bound


def simulate(NT, R, CB, J, S):
    G = J * NT
    seq = []              # op tags in issue order
    seq += [("Q", 0)] * 4
    for g in range(R - CB):
        seq.append(("P", g))
    ngroups = (G + CB - 1) // CB
    for s in range(ngroups):
        gl = s * CB + CB - 1
        need = max(i for i, t in enumerate(seq) if t == ("P", gl))
        k = len(seq) - 1 - need
        assert k == ring_wait_count(s, NT, R, CB, S), (NT, R, CB, J, S, s, k, ring_wait_count(s, NT, R, CB, S))
        for g in range(s * CB + R - CB, s * CB + R):      # refill after the barrier
            seq.append(("P", g))
        for g in range(s * CB, min(s * CB + CB, G)):       # compute; unit boundary after the unit's last chunk
            if g % NT == NT - 1:
                seq += [("Q", g // NT + 1)] * 4 + [("S", g // NT)] * S
            # (the Q wait at the boundary is wave-local: vmcnt(S))
    return True


if __name__ == "__main__":
    n = 0
    for NT, R, CB, J, S in itertools.product(range(1, 9), range(2, 11), range(1, 6), range(1, 6), (0, 4, 5)):
        if R < 2 * CB:
            continue
        simulate(NT, R, CB, J, S)
        n += 1
    print(f"ok: {n} configurations")
