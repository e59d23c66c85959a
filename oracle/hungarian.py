"""oracle/hungarian.py -- TEST INFRASTRUCTURE ONLY: the checker of the device matching in
bcm3_amd/csrc/cellpop_kernels.hip (cp_timecourse_kernel). Nothing in the product path imports it.

Restatement of the assignment routine the reference's cell-population time-course likelihood calls
(DataLikelihoodTimeCourse.cpp:323): hungarianMinimumWeightPerfectMatching of the third-party
"hungarian2" (James Payor, December 2017, MIT licence), vendored in the reference at
dependencies/hungarian2/hungarian.cpp with one BCM change (an explicit right-node count and edge
count, changes_for_bcm.txt). It cannot be built here: it includes the reference's Utils.h, which
needs Boost. The restatement follows it statement for statement, because its result is not always
the minimum-weight matching and the likelihood is the sum over the matching it returns:

  * hungarian.cpp:167 stores the initial reduced cost in an `int` before the tightness test
    `< 1e-12`, so every edge whose reduced cost truncates to 0 (anything below 1.0) starts "tight",
    and the greedy initial matching (:192-203) may take it. A reduced cost outside int's range
    converts to INT_MIN on x86-64 (cvttsd2si) and is tight as well. `_tight0` restates both.
  * the breadth-first search (:292-329) keeps scanning a node's tight edges after it has found an
    unmatched right node, so the LAST such node of the scan ends the search;
  * tight edges that have gone loose are swapped to the end of the tight prefix (:306-311), and the
    slack cache keeps edge indices that later swaps may have moved (:353, :413-421).

Pinned against the dependency's own test (dependencies/hungarian2/test.cpp:45-80: agreement with
brute force on random graphs with integer costs 0..6, where the int truncation is exact) by
tests/test_timecourse.py, which also holds hand-made cases of the quirks above."""
import sys
from collections import deque

OO = sys.float_info.max  # std::numeric_limits<Real>::max() (hungarian.cpp:25)
UNMATCHED = -1


def _tight0(reduced):
    """(int)reduced < 1e-12 with x86-64 conversion semantics (hungarian.cpp:167-169)"""
    if not (-2147483649.0 < reduced < 2147483648.0):  # NaN or out of range -> INT_MIN
        return True
    return int(reduced) < 1e-12  # int() truncates toward zero like the C conversion


def min_weight_perfect_matching(n, n_right, edges):
    """edges: sequence of (left, right, cost) in the caller's order. Returns the list of right
    nodes matched to left nodes 0..n-1, or [] when the routine finds no perfect matching."""
    # per-node edge counts; a node with no edge -> no matching (hungarian.cpp:52-77)
    lcount = [0] * n
    rcount = [0] * n
    for l, r, _ in edges:
        if 0 <= l < n:
            lcount[l] += 1
        if 0 <= r < n:
            rcount[r] += 1
    for i in range(n):
        if lcount[i] == 0 or rcount[i] == 0:
            return []
    # edge lists of the left nodes, sorted by (right, cost), first of each right kept (:79-106)
    adj = [[] for _ in range(n)]
    for l, r, c in edges:
        if 0 <= l < n and 0 <= r < n:
            adj[l].append((r, c))
    for i in range(n):
        adj[i].sort()
        kept = []
        for r, c in adj[i]:
            if not kept or kept[-1][0] != r:
                kept.append((r, c))
        adj[i] = kept
    # potentials (:122-148): left = smallest incident cost, right = smallest reduced cost over ALL edges
    lpot = []
    for i in range(n):
        m = adj[i][0][1]
        for _, c in adj[i][1:]:
            if c < m:
                m = c
        lpot.append(m)
    rpot = [OO] * n_right
    for l, r, c in edges:
        red = c - lpot[l]
        if rpot[r] > red:
            rpot[r] = red
    # tight prefix of each edge list (:162-177)
    ntight = [0] * n
    for i in range(n):
        a = adj[i]
        t = 0
        for k in range(len(a)):
            r, c = a[k]
            if _tight0(c - lpot[i] - rpot[r]):
                if k != t:
                    a[t], a[k] = a[k], a[t]
                t += 1
        ntight[i] = t
    # greedy initial matching over tight edges (:185-209)
    lmatch = [UNMATCHED] * n
    rmatch = [UNMATCHED] * n
    card = 0
    for i in range(n):
        for k in range(ntight[i]):
            j = adj[i][k][0]
            if rmatch[j] == UNMATCHED:
                card += 1
                rmatch[j] = i
                lmatch[i] = j
                break
    if card == n:
        return lmatch

    while card < n:
        slack = [OO] * n
        slack_from = [UNMATCHED] * n
        slack_edge = [0] * n
        queue = deque()
        seen = [False] * n
        back = [UNMATCHED] * n
        # unmatched left node with the fewest tight edges, first on ties (:269-277)
        start, fewest = UNMATCHED, OO
        for i in range(n):
            if lmatch[i] == UNMATCHED and ntight[i] < fewest:
                fewest = ntight[i]
                start = i
        queue.append(start)
        seen[start] = True
        end = UNMATCHED
        while end == UNMATCHED:
            while end == UNMATCHED and queue:
                i = queue.popleft()
                a = adj[i]
                k = 0
                while k < ntight[i]:
                    j, c = a[k]
                    if c > lpot[i] + rpot[j]:  # gone loose: swap behind the tight prefix (:306-311)
                        ntight[i] -= 1
                        a[k], a[ntight[i]] = a[ntight[i]], a[k]
                        continue
                    if back[j] == UNMATCHED:
                        back[j] = i
                        m = rmatch[j]
                        if m == UNMATCHED:
                            end = j  # the scan goes on: the last unmatched node wins
                        elif not seen[m]:
                            seen[m] = True
                            queue.append(m)
                    k += 1
                if end == UNMATCHED:  # slack of the non-tight edges to unreached right nodes (:336-357)
                    p = lpot[i]
                    for k in range(ntight[i], len(a)):
                        j, c = a[k]
                        if rmatch[j] == UNMATCHED or not seen[rmatch[j]]:
                            red = c - p - rpot[j]
                            if red < slack[j]:
                                slack[j] = red
                                slack_from[j] = i
                                slack_edge[j] = k
            if end == UNMATCHED:
                # smallest slack over unreached right nodes, first on ties (:372-389)
                jmin, smin = UNMATCHED, OO
                for j in range(n):
                    if rmatch[j] == UNMATCHED or not seen[rmatch[j]]:
                        if slack[j] < smin:
                            smin = slack[j]
                            jmin = j
                if jmin == UNMATCHED or slack_from[jmin] == UNMATCHED:
                    return []
                for i in range(n):  # (:396-403)
                    if seen[i]:
                        lpot[i] += smin
                        if lmatch[i] != UNMATCHED:
                            rpot[lmatch[i]] -= smin
                for j in range(n):  # (:406-444)
                    if rmatch[j] == UNMATCHED or not seen[rmatch[j]]:
                        slack[j] -= smin
                        if slack[j] == 0:
                            i = slack_from[j]
                            k = slack_edge[j]
                            a = adj[i]
                            if k != ntight[i]:
                                a[k], a[ntight[i]] = a[ntight[i]], a[k]
                            ntight[i] += 1
                            if end == UNMATCHED:
                                back[j] = i
                                m = rmatch[j]
                                if m == UNMATCHED:
                                    end = j
                                elif not seen[m]:
                                    seen[m] = True
                                    queue.append(m)
        card += 1
        j = end  # flip the augmenting path (:457-468)
        while j != UNMATCHED:
            i = back[j]
            nxt = lmatch[i]
            rmatch[j] = i
            lmatch[i] = j
            j = nxt
    return lmatch


def brute_force(n, edges):
    """the dependency's own ground truth (test.cpp:7-43): the cheapest perfect matching by
    exhaustive search over the edges in order, strict improvement only"""
    lm = [False] * n
    rm = [False] * n

    def rec(start, count):
        if count == n:
            return 0.0, []
        best, best_edges = float(1 << 20), []
        for k in range(start, len(edges)):
            l, r, c = edges[k]
            if not lm[l] and not rm[r]:
                lm[l] = rm[r] = True
                sub, se = rec(k + 1, count + 1)
                lm[l] = rm[r] = False
                if sub + c < best:
                    best = sub + c
                    best_edges = se + [k]
        return best, best_edges

    _, chosen = rec(0, 0)
    out = [0] * n
    for k in chosen:
        out[edges[k][0]] = edges[k][1]
    return out
