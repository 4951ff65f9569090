"""TEST INFRASTRUCTURE: numpy statement of the contact-form level-0 repair over the friction pyramid
(the algorithm of qppvm_amd/csrc/fric_lsi.h, used by contact_kernel.hip:contact_level0 with mu > 0),
checked against the oracle's level 0 (oracle/wbq_oracle_contact.c:wbq_ref_contact_one, a 1e-10-ridge
QP in x-space) and used by tests/test_kkt_oracle.py to pin the LSI certificate (tests/kkt.py).

Level 0 in z = (tau_a, w) space (contact_kernel.hip): min 0.5 ||A0 z - b||^2 over
  lo <= z <= hi (torque and wrench boxes), s f_x - mu f_z <= 0, s f_y - mu f_z <= 0 per active contact.
A primal active set in the BVLS pattern (Stark-Parker): single variables carry box states as BVLS;
the three force components of an active contact form a group whose active constraints (box sides
and pyramid faces) define a projector P_c onto the free directions. Inner loop: minimum-norm LS
step dz = P A0^T w with (A0 P A0^T) w = b - A0 z, interpolated back at the first blocking
constraint; outer loop: multipliers (single variables: w_j; groups: lambda = -(N^T N)^-1 N^T g),
release the most violated one.

    python tests/fric_lsi_ref.py [mu ...]   (the comparison with the oracle over the repair sweep)
"""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tests/", 1)[0])
import oracle  # noqa: E402
from qppvm_amd.problem import ContactProblem  # noqa: E402
from qppvm_amd.synth import contact_instances  # noqa: E402

MASKS4 = [0b0011, 0b0111, 0b1111, 0b0101, 0b1010, 0b1100]


def face_normal(k, mu):
    v = np.zeros(3)
    v[k >> 1] = -1.0 if (k & 1) else 1.0
    v[2] = -mu
    return v


def group_normals(st3, fm, mu):
    """active normals (outward) of a contact: box sides then faces; codes (0..2 box comp, 3..6 face)"""
    N, codes = [], []
    for k in range(3):
        if st3[k] != 0:
            e = np.zeros(3)
            e[k] = 1.0 if st3[k] > 0 else -1.0
            N.append(e)
            codes.append(k)
    for k in range(4):
        if (fm >> k) & 1:
            N.append(face_normal(k, mu))
            codes.append(3 + k)
    return (np.array(N).reshape(-1, 3), codes)


def projector(N):
    P = np.eye(3)
    Q = []
    for nv in N:
        v = nv.copy()
        for _ in range(2):
            for q in Q:
                v -= q * (q @ v)
        nn = np.linalg.norm(v)
        if nn > 1e-12 * np.linalg.norm(nv):
            Q.append(v / nn)
    for q in Q:
        P -= np.outer(q, q)
    return P


def minnorm(G, r, tol=1e-12):
    """min-norm LS weights of G w = r (G PSD 6x6), by eigen-decomposition (the kernel: PivChol)."""
    ev, V = np.linalg.eigh(G)
    keep = ev > tol * max(ev.max(), 1e-300)
    return V[:, keep] @ ((V[:, keep].T @ r) / ev[keep])


def lsi_level0(A, b, lo, hi, groups, mu, maxit=2000):
    """A [6][nz]; groups: list of (i0) start index of an active contact's (fx, fy, fz)"""
    nz = A.shape[1]
    z = np.clip(np.zeros(nz), lo, hi)
    st = np.zeros(nz, dtype=int)
    st[lo == hi] = -1
    fm = {g: 0 for g in groups}
    ingroup = np.zeros(nz, dtype=bool)
    for g in groups:
        ingroup[g:g + 3] = True
    abm = max(1.0, np.abs(A.T @ b).max())
    it = 0
    excl = None  # (kind, idx, code)
    freed = None
    while True:
        while True:
            it += 1
            P = np.zeros((nz, nz))
            for j in range(nz):
                if not ingroup[j]:
                    P[j, j] = 1.0 if st[j] == 0 else 0.0
            for g in groups:
                N, _ = group_normals(st[g:g + 3], fm[g], mu)
                P[g:g + 3, g:g + 3] = projector(N)
            if np.abs(P).max() == 0:
                break
            r = b - A @ z
            G = A @ P @ A.T
            w = minnorm(G, r)
            dz = P @ (A.T @ w)
            # ratio test
            best, blk = np.inf, None
            for j in range(nz):
                if st[j] != 0 or lo[j] == hi[j]:
                    continue
                if dz[j] > 0 and z[j] + dz[j] > hi[j]:
                    a = (hi[j] - z[j]) / dz[j]
                    if a < best:
                        best, blk = a, ("box", j, 1)
                elif dz[j] < 0 and z[j] + dz[j] < lo[j]:
                    a = (lo[j] - z[j]) / dz[j]
                    if a < best:
                        best, blk = a, ("box", j, -1)
            for g in groups:
                for k in range(4):
                    if (fm[g] >> k) & 1:
                        continue
                    nv = face_normal(k, mu)
                    ph, dph = nv @ z[g:g + 3], nv @ dz[g:g + 3]
                    if dph > 0 and ph + dph > 0:
                        a = max(0.0, -ph) / dph
                        if a < best:
                            best, blk = a, ("face", g, k)
            if blk is None or best >= 1.0:
                z = z + dz
                freed = None
                excl = None
                break
            alpha = max(best, 0.0)
            if freed is not None and blk == freed and alpha == 0.0:
                # the constraint just released wants back in: re-add, exclude
                if blk[0] == "box":
                    st[blk[1]] = blk[2]
                    z[blk[1]] = hi[blk[1]] if blk[2] > 0 else lo[blk[1]]
                else:
                    fm[blk[1]] |= 1 << blk[2]
                excl = blk
                freed = None
                break
            excl = None
            z = z + alpha * dz
            if blk[0] == "box":
                st[blk[1]] = blk[2]
                z[blk[1]] = hi[blk[1]] if blk[2] > 0 else lo[blk[1]]
            else:
                fm[blk[1]] |= 1 << blk[2]
            freed = None
            if it >= maxit:
                break
        # KKT: w = A^T (b - A z) = -grad
        wv = A.T @ (b - A @ z)
        wx = np.abs(A.T @ (A @ z)).max()
        wtol = 1e-11 * max(abm, wx)
        bestv, cand = -np.inf, None
        for j in range(nz):
            if ingroup[j] or st[j] == 0 or lo[j] == hi[j]:
                continue
            v = wv[j] if st[j] < 0 else -wv[j]
            if ("box", j, st[j]) == excl:
                continue
            if v > bestv:
                bestv, cand = v, ("box", j, st[j])
        lam_all = {}
        for g in groups:
            N, codes = group_normals(st[g:g + 3], fm[g], mu)
            if len(codes) == 0:
                continue
            gr = -wv[g:g + 3]
            lam = -np.linalg.solve(N @ N.T, N @ gr)
            for c, l, nv in zip(codes, lam, N):
                key = ("box", g + c, st[g + c]) if c < 3 else ("face", g, c - 3)
                lam_all[key] = l
                v = -l * np.linalg.norm(nv)
                if key == excl:
                    continue
                if v > bestv:
                    bestv, cand = v, key
        if cand is None or not (bestv > wtol):
            break
        if it >= maxit:
            return z, st, fm, it, True, None
        if cand[0] == "box":
            st[cand[1]] = 0
        else:
            fm[cand[1]] &= ~(1 << cand[2])
        freed = cand
    # multipliers at the optimum (pins)
    wv = A.T @ (b - A @ z)
    pins = {}
    for j in range(nz):
        if not ingroup[j] and st[j] != 0 and lo[j] != hi[j]:
            pins[("box", j, st[j])] = wv[j] if st[j] < 0 else -wv[j]
    for g in groups:
        N, codes = group_normals(st[g:g + 3], fm[g], mu)
        if codes:
            lam = -np.linalg.solve(N @ N.T, N @ (-wv[g:g + 3]))
            for c, l in zip(codes, lam):
                pins[("box", g + c, st[g + c]) if c < 3 else ("face", g, c - 3)] = l
    return z, st, fm, it, False, pins


def zspace(prob, inp, b):
    n, nc, wd = prob.n, prob.nc, prob.wrench_dim
    M, h, Jw, Jc = inp["M"][b], inp["h"][b], inp["Jw"][b], inp["Jc"][b]
    W = np.linalg.solve(M, Jw.T)  # n x 6
    L = oracle.contact_assemble(prob, inp, b)
    bw = L["bw"]
    na = n - 6
    cols = [W[6 + a] for a in range(na)]
    cm = int(inp["cmask"][b])
    lo, hi = [], []
    for a in range(na):
        lo.append(prob.tau_min[6 + a] if prob.torque_rows else -np.inf)
        hi.append(prob.tau_max[6 + a] if prob.torque_rows else np.inf)
    groups = []
    flb = list(prob.f_lb) + list(prob.m_lb)
    fub = list(prob.f_ub) + list(prob.m_ub)
    for c in range(nc):
        on = (cm >> c) & 1
        if on and prob.mu > 0:
            groups.append(na + wd * c)
        for k in range(wd):
            cols.append(W.T @ Jc[c, k])
            lo.append(flb[k] if on else 0.0)
            hi.append(fub[k] if on else 0.0)
    A = np.array(cols).T
    return A, bw + W.T @ h, np.array(lo), np.array(hi), groups, W.T @ h


def main():
    mus = [float(a) for a in sys.argv[1:]] or [0.3, 0.5]
    for mu in mus:
        tot = dict(rep=0, bad=0, capped=0, maxit=0)
        worst = 0.0
        for seed in range(100, 120):
            n, nc = 12, 4
            free = ContactProblem(n=n, nc=nc, mu=mu)
            inp = contact_instances(free, 64, seed=seed, masks=MASKS4)
            tf = oracle.contact_batch(free, inp)[0]
            prob = ContactProblem(n=n, nc=nc, mu=mu, torque_rows=True,
                                  tau_max=float(np.quantile(np.abs(tf[:, 6:]), 0.4)))
            tau_r, x_r, st_r, _, rep = oracle.contact_batch(prob, inp)
            for b in np.where((st_r == 0) & (rep != 0))[0]:
                A, bb, lo, hi, groups, wth = zspace(prob, inp, b)
                z, st, fm, it, capped, pins = lsi_level0(A, bb, lo, hi, groups, mu)
                y = A @ z - wth
                yr = inp["Jw"][b] @ x_r[b, :n]
                e = np.abs(y - yr).max() / max(1.0, np.abs(yr).max())
                worst = max(worst, e)
                tot["rep"] += 1
                tot["maxit"] = max(tot["maxit"], it)
                tot["capped"] += int(capped)
                if e > 1e-7:
                    tot["bad"] += 1
                    if tot["bad"] <= 5:
                        print("mismatch", seed, b, e, it)
        print(f"mu={mu}: {tot}, worst y0* rel err {worst:.2e}")


if __name__ == "__main__":
    main()


def check_obj(seed, b, mu):
    n, nc = 12, 4
    free = ContactProblem(n=n, nc=nc, mu=mu)
    inp = contact_instances(free, 64, seed=seed, masks=MASKS4)
    tf = oracle.contact_batch(free, inp)[0]
    prob = ContactProblem(n=n, nc=nc, mu=mu, torque_rows=True, tau_max=float(np.quantile(np.abs(tf[:, 6:]), 0.4)))
    tau_r, x_r, st_r, _, rep = oracle.contact_batch(prob, inp)
    A, bb, lo, hi, groups, wth = zspace(prob, inp, b)
    z, st, fm, it, capped, pins = lsi_level0(A, bb, lo, hi, groups, mu)
    yr = inp["Jw"][b] @ x_r[b, :n]
    print("obj mine", 0.5 * np.sum((A @ z - bb) ** 2), "oracle", 0.5 * np.sum((yr + wth - bb) ** 2),
          "|z|", np.abs(z).max(), "pins", {k: round(v, 6) for k, v in pins.items()})


def level1_check(mus=(0.3, 0.5), seeds=range(100, 120), pin=True):
    """full pipeline: level-0 emulation, then the oracle's dual QP on level 1 with y0* and the pins"""
    for mu in mus:
        worst, nbad, nrep = 0.0, 0, 0
        for seed in seeds:
            n, nc = 12, 4
            free = ContactProblem(n=n, nc=nc, mu=mu)
            inp = contact_instances(free, 64, seed=seed, masks=MASKS4)
            tf = oracle.contact_batch(free, inp)[0]
            prob = ContactProblem(n=n, nc=nc, mu=mu, torque_rows=True,
                                  tau_max=float(np.quantile(np.abs(tf[:, 6:]), 0.4)))
            tau_r, x_r, st_r, _, rep = oracle.contact_batch(prob, inp)
            wd, na = prob.wrench_dim, n - 6
            for b in np.where((st_r == 0) & (rep != 0))[0]:
                A, bb, lo, hi, groups, wth = zspace(prob, inp, b)
                z, st, fm, it, capped, pins = lsi_level0(A, bb, lo, hi, groups, mu)
                y = A @ z - wth
                L = oracle.contact_assemble(prob, inp, b)
                e = L["e"].copy()
                e[:6] = y
                clo, chi = L["clo"].copy(), L["chi"].copy()
                abm = max(1.0, np.abs(A.T @ bb).max())
                if pin:
                    for key, v in pins.items():
                        lam = -v if key[0] == "box" and key[1] not in [gg + k for gg in groups for k in range(3)] else v
                        if lam <= 1e-9 * abm:
                            continue
                        if key[0] == "box":
                            j, s = key[1], key[2]
                            row = (j - na) if j >= na else wd * nc + 4 * nc + j
                            if s > 0:
                                clo[row] = chi[row]
                            else:
                                chi[row] = clo[row]
                        else:
                            c = (key[1] - na) // wd
                            clo[wd * nc + 4 * c + key[2]] = 0.0
                x, s1, _ = oracle.dual_qp(L["H"], L["g"], L["E"], e, L["C"], clo, chi)
                nrep += 1
                if s1 != 0:
                    nbad += 1
                    print("level-1 status", s1, seed, b)
                    continue
                M, h, Jc = inp["M"][b], inp["h"][b], inp["Jc"][b]
                tau = M @ x[:n] + h
                for c in range(nc):
                    tau -= Jc[c, :wd].T @ x[n + wd * c:n + wd * (c + 1)]
                err = np.abs(tau - tau_r[b]).max() / max(1.0, np.abs(tau_r[b]).max())
                worst = max(worst, err)
                if err > 1e-6:
                    nbad += 1
                    print("tau mismatch", seed, b, err)
        print(f"mu={mu}: repaired {nrep}, bad {nbad}, worst tau rel err {worst:.2e}")
