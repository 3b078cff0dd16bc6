"""The persistent Cholesky's worker claim order (kernels/chol.hip task_of / task_local) restated
in Python, and a claim-queue simulation of the persistent launch: workers claim task indices in
order, each waits until its dependencies are published (the spin waits of k_chol_persist), and
the diagonal chain steps when its two tiles are ready.  Checks that the claim order is a
permutation of the step tasks and that every order the library uses drains -- step order with any
worker count, order 1 with more workers than one critical set holds (4 tasks, 6 with the split
critical updates; the kernel falls back to step order below that)."""
import pytest


def step_tasks(R, split):
    return R + R * (R + 1) // 2 - 1 + (2 if split and R >= 2 else 0)


def task_local(k, l, T, split, rowmajor=False):
    R = T - 1 - k
    if l < R:
        return (k, k + 1 + l, -1, -1)
    q = l - R
    if split and R >= 2:
        if q < 4:
            return (k, k + 2, k + 1 if q < 2 else k + 2, q & 1)
        q -= 2
    if rowmajor and q >= 2:
        r, i = q - 2, k + 3
        while r >= i - k:
            r -= i - k
            i += 1
        return (k, i, k + 1 + r, -1)
    u = 1 if q == 0 else (R if q == 1 else (q if q < R else q + 1))
    j = k + 1
    while u >= T - j:
        u -= T - j
        j += 1
    return (k, j + u, j, -1)


def task_of(g, T, order, split, rowmajor=False):
    if order == 1:
        nc = 6 if split else 4
        csz = lambda kk: nc if T - 1 - kk >= 2 else 1
        cmap = lambda x, RR: x if x < 2 else RR + x - 2
        if g < csz(0):
            return task_local(0, cmap(g, T - 1), T, split, rowmajor)
        g -= csz(0)
        kk = 0
        while True:
            if kk + 1 <= T - 2:
                c1 = csz(kk + 1)
                if g < c1:
                    return task_local(kk + 1, cmap(g, T - 2 - kk), T, split, rowmajor)
                g -= c1
            RR = T - 1 - kk
            S = step_tasks(RR, split)
            rest = S - csz(kk)
            if g < rest or kk >= T - 2:
                return task_local(kk, g + 2 if g < RR - 2 else g + (6 if split and RR >= 2 else 4), T, split, rowmajor)
            g -= rest
            kk += 1
    k, R = 0, T - 1
    while True:
        S = step_tasks(R, split)
        if g < S or R <= 1:
            break
        g -= S
        k += 1
        R -= 1
    return task_local(k, g, T, split, rowmajor)


def all_tasks(T, split):
    return [(k, *task_local(k, l, T, split)[1:]) for k in range(T - 1) for l in range(step_tasks(T - 1 - k, split))]


def simulate(T, workers, order, split, selfl=True, rowmajor=False):
    """True when every task and chain step completes (no state in which every worker waits on a
    task nobody can run)."""
    ntasks = sum(step_tasks(R, split) for R in range(T - 1, 0, -1))
    ver = {(i, j): 0 for i in range(T) for j in range(i + 1)}   # tile versions (steps applied)
    halves = {}
    lcnt = [0] * T   # panel row i's L published through step lcnt - 1
    bcnt = [0] * T   # b_i's updates through step bcnt - 1
    wdone = [False] * T
    d_next = 1       # the chain factors tile 0 itself first (the reducing form)
    wdone[0] = True
    nxt = 0
    held = [None] * workers

    def ready(t):
        k, i, j, h = t
        if j < 0:   # panel row i of step k
            return ver[(i, k)] >= k and bcnt[k] >= k and bcnt[i] >= k and wdone[k]
        if h >= 0 or (selfl and i == k + 2 and j >= k + 1):   # forms L_ik, L_jk itself
            return ver[(i, j)] >= k and ver[(i, k)] >= k and ver[(j, k)] >= k and wdone[k]
        return ver[(i, j)] >= k and lcnt[i] >= k + 1 and lcnt[j] >= k + 1

    def run(t):
        k, i, j, h = t
        if j < 0:
            lcnt[i] = k + 1
            bcnt[i] = k + 1
        elif h >= 0:
            halves[(i, j, k)] = halves.get((i, j, k), 0) + 1
            if halves[(i, j, k)] == 2:
                ver[(i, j)] = k + 1
        else:
            ver[(i, j)] = k + 1

    done = 0
    while done < ntasks or d_next < T:
        progress = False
        # the chain: step d needs tiles (d, d-1) and (d, d) through step d-2, and W_{d-1}
        if d_next < T and wdone[d_next - 1] and ver[(d_next, d_next - 1)] >= d_next - 1 and \
                ver[(d_next, d_next)] >= d_next - 1:
            ver[(d_next, d_next)] = d_next   # its own last update (the prepare)
            wdone[d_next] = True
            d_next += 1
            progress = True
        for w in range(workers):
            if held[w] is None and nxt < ntasks:
                held[w] = task_of(nxt, T, order, split, rowmajor)
                nxt += 1
                progress = True
            if held[w] is not None and ready(held[w]):
                run(held[w])
                held[w] = None
                done += 1
                progress = True
        if not progress:
            return False
    return True


@pytest.mark.parametrize("split,rowmajor", [(False, False), (True, False), (True, True), (False, True)])
def test_claim_order_is_a_permutation(split, rowmajor):
    for T in range(2, 36):
        nt = sum(step_tasks(R, split) for R in range(T - 1, 0, -1))
        for order in (0, 1):
            got = sorted(task_of(g, T, order, split, rowmajor) for g in range(nt))
            assert got == sorted(all_tasks(T, split)), (T, order)


@pytest.mark.parametrize("split,rowmajor", [(False, False), (True, False), (True, True), (False, True)])
def test_claim_orders_drain(split, rowmajor):
    need = 7 if split else 5   # order 1 needs more workers than one critical set holds
    for T in (2, 3, 4, 5, 8, 17, 33):
        for workers in (1, 2, 3, need - 1, need, need + 1, 16, 64):
            assert simulate(T, workers, 0, split, rowmajor=rowmajor), ("step order", T, workers)
            if workers >= need:
                assert simulate(T, workers, 1, split, rowmajor=rowmajor), ("order 1", T, workers)


def test_order1_needs_the_worker_guard():
    """The model has teeth: with fewer workers than a critical set's waiting tasks order 1 stalls
    (why k_chol_persist claims in step order below 6 / 8 workers)."""
    assert not simulate(8, 3, 1, False)
    assert not simulate(8, 5, 1, True)
