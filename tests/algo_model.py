"""Executable model of the HIP kernels' algorithm (test helper, fp64 torch).

This is NOT the oracle: it restates, in vectorised torch, exactly the
restructured arithmetic the HIP kernels execute, with a hand-written backward,
so the algebra can be checked against the oracle's autograd on the CPU before
(and while) debugging the kernels:

* token pruning: only query row 0 (agent) / the last A+3 rows (mixer) are
  propagated through the blocks (keys never change, transformer.py:140);
* folded projections: per head M_h = Wk_hᵀ·Wq_h/√E (scores = (M_h x)·key) and
  N_h = U_h·Wv_h (attended = Σ_h N_h z_h + b_U), so K/V are never formed;
* agent attention in observation space: entity keys are We·o_j + b_e, so
  scores use w_h = We_ᵀ·u_h (F-dim) and z_h = p_0 h + We·ô_h + P_h b_e.
"""
import math

import torch
import torch.nn.functional as F


def derive(p, pre, E, H, D):
    """Folded per-block weights from the reference parameters."""
    out = []
    s = 1.0 / math.sqrt(E)
    for d in range(D):
        b = f"{pre}tblocks.{d}."
        Wq = p[b + "attention.toqueries.weight"].view(H, E, E)
        Wk = p[b + "attention.tokeys.weight"].view(H, E, E)
        Wv = p[b + "attention.tovalues.weight"].view(H, E, E)
        U = p[b + "attention.unifyheads.weight"].view(E, H, E)
        M = torch.einsum("hmi,hmk->hik", Wk, Wq) * s          # [H,E,E]
        N = torch.einsum("ohm,hmk->ohk", U, Wv).reshape(E, H * E)  # [E,H*E]
        out.append(dict(M=M.reshape(H * E, E), N=N, bu=p[b + "attention.unifyheads.bias"],
                        g1=p[b + "norm1.weight"], n1=p[b + "norm1.bias"],
                        W1=p[b + "ff.0.weight"], c1=p[b + "ff.0.bias"],
                        W2=p[b + "ff.2.weight"], c2=p[b + "ff.2.bias"],
                        g2=p[b + "norm2.weight"], n2=p[b + "norm2.bias"]))
    return out


def fold_grads(p, pre, E, H, D, gblocks):
    """Map grads of (M, N) back to (Wq, Wk, Wv, U)."""
    s = 1.0 / math.sqrt(E)
    g = {}
    for d in range(D):
        b = f"{pre}tblocks.{d}."
        Wq = p[b + "attention.toqueries.weight"].view(H, E, E)
        Wk = p[b + "attention.tokeys.weight"].view(H, E, E)
        Wv = p[b + "attention.tovalues.weight"].view(H, E, E)
        U = p[b + "attention.unifyheads.weight"].view(E, H, E)
        gM = gblocks[d]["M"].view(H, E, E)
        gN = gblocks[d]["N"].view(E, H, E)
        g[b + "attention.toqueries.weight"] = (torch.einsum("hmi,hik->hmk", Wk, gM) * s).reshape(H * E, E)
        g[b + "attention.tokeys.weight"] = (torch.einsum("hmk,hik->hmi", Wq, gM) * s).reshape(H * E, E)
        g[b + "attention.tovalues.weight"] = torch.einsum("ohm,ohk->hmk", U, gN).reshape(H * E, E)
        g[b + "attention.unifyheads.weight"] = torch.einsum("ohk,hmk->ohm", gN, Wv).reshape(E, H * E)
        for k_src, k_dst in [("bu", "attention.unifyheads.bias"), ("g1", "norm1.weight"),
                             ("n1", "norm1.bias"), ("W1", "ff.0.weight"), ("c1", "ff.0.bias"),
                             ("W2", "ff.2.weight"), ("c2", "ff.2.bias"), ("g2", "norm2.weight"),
                             ("n2", "norm2.bias")]:
            g[b + k_dst] = gblocks[d][k_src]
    return g


def _ln(r, g, n, eps=1e-5):
    mu = r.mean(-1, keepdim=True)
    var = ((r - mu) ** 2).mean(-1, keepdim=True)
    rstd = 1.0 / torch.sqrt(var + eps)
    xh = (r - mu) * rstd
    return xh * g + n, xh, rstd


def _ln_bwd(gout, xh, rstd, g):
    gxh = gout * g
    return rstd * (gxh - gxh.mean(-1, keepdim=True) - xh * (gxh * xh).mean(-1, keepdim=True))


def _ffn_ln_fwd(bk, a, x):
    y, xh1, rs1 = _ln(a + x, bk["g1"], bk["n1"])
    f1 = y @ bk["W1"].T + bk["c1"]
    f1r = torch.relu(f1)
    f = f1r @ bk["W2"].T + bk["c2"]
    xo, xh2, rs2 = _ln(f + y, bk["g2"], bk["n2"])
    return xo, dict(y=y, xh1=xh1, rs1=rs1, f1=f1, f1r=f1r, xh2=xh2, rs2=rs2)


def _ffn_ln_bwd(bk, c, gx, gb):
    gb["g2"] += (gx * c["xh2"]).sum(0)
    gb["n2"] += gx.sum(0)
    gr2 = _ln_bwd(gx, c["xh2"], c["rs2"], bk["g2"])
    gb["W2"] += gr2.T @ c["f1r"]
    gb["c2"] += gr2.sum(0)
    gf1 = (gr2 @ bk["W2"]) * (c["f1"] > 0)
    gb["W1"] += gf1.T @ c["y"]
    gb["c1"] += gf1.sum(0)
    gy = gr2 + gf1 @ bk["W1"]
    gb["g1"] += (gy * c["xh1"]).sum(0)
    gb["n1"] += gy.sum(0)
    return _ln_bwd(gy, c["xh1"], c["rs1"], bk["g1"])  # = ga = grad wrt (a + x)


def _zero_gblocks(blocks):
    return [{k: torch.zeros_like(v) for k, v in bk.items()} for bk in blocks]


# ----------------------------------------------------------------------------- agent
def agent_step_fwd(W, h, o, H):
    """One agent step for R rows. h [R,E], o [R,n,F]. Returns (q, h', cache)."""
    R, E = h.shape
    We, be = W["We"], W["be"]
    x = h
    caches = []
    for bk in W["blocks"]:
        u = (x @ bk["M"].T).view(R, H, E)
        w = u @ We                                   # [R,H,F]  (We^T u)
        c = u @ be                                   # [R,H]
        s0 = (u * h[:, None, :]).sum(-1)             # [R,H]
        sj = torch.einsum("rhf,rjf->rhj", w, o) + c[..., None]
        s = torch.cat([s0[..., None], sj], -1)       # [R,H,1+n]
        pr = torch.softmax(s, -1)
        p0, pj = pr[..., 0], pr[..., 1:]
        oh = torch.einsum("rhj,rjf->rhf", pj, o)     # [R,H,F]
        P = pj.sum(-1)                               # [R,H]
        z = p0[..., None] * h[:, None, :] + oh @ We.T + P[..., None] * be
        a = z.reshape(R, H * E) @ bk["N"].T + bk["bu"]
        xo, cc = _ffn_ln_fwd(bk, a, x)
        cc.update(x=x, u=u, w=w, pr=pr, oh=oh, P=P, z=z)
        caches.append(cc)
        x = xo
    q = x @ W["Wo"].T + W["bo"]
    return q, x, caches


def agent_step_bwd(W, h, o, H, hout, caches, gh, gq, g):
    """Backward of agent_step_fwd; accumulates into g, returns grad wrt h."""
    R, E = h.shape
    We, be = W["We"], W["be"]
    g["Wo"] += gq.T @ hout
    g["bo"] += gq.sum(0)
    gx = gh + gq @ W["Wo"]
    gh_in = torch.zeros_like(h)
    for d in reversed(range(len(W["blocks"]))):
        bk, c, gb = W["blocks"][d], caches[d], g["blocks"][d]
        ga = _ffn_ln_bwd(bk, c, gx, gb)
        gx_prev = ga.clone()
        gb["N"] += ga.T @ c["z"].reshape(R, H * E)
        gb["bu"] += ga.sum(0)
        gz = (ga @ bk["N"]).view(R, H, E)
        pr, u, w, oh, P = c["pr"], c["u"], c["w"], c["oh"], c["P"]
        p0, pj = pr[..., 0], pr[..., 1:]
        gp0 = (gz * h[:, None, :]).sum(-1)
        gh_in += (p0[..., None] * gz).sum(1)
        goh = gz @ We                                # [R,H,F]
        g["We"] += torch.einsum("rhe,rhf->ef", gz, oh)
        gP = gz @ be
        g["be"] += (P[..., None] * gz).sum((0, 1))
        gpj = torch.einsum("rhf,rjf->rhj", goh, o) + gP[..., None]
        gp = torch.cat([gp0[..., None], gpj], -1)
        gs = pr * (gp - (pr * gp).sum(-1, keepdim=True))
        gs0, gsj = gs[..., 0], gs[..., 1:]
        gu = gs0[..., None] * h[:, None, :]
        gh_in += (gs0[..., None] * u).sum(1)
        gw = torch.einsum("rhj,rjf->rhf", gsj, o)
        gc = gsj.sum(-1)
        gu = gu + gw @ We.T + gc[..., None] * be
        g["We"] += torch.einsum("rhe,rhf->ef", u, gw)
        g["be"] += (gc[..., None] * u).sum((0, 1))
        gu = gu.reshape(R, H * E)
        gb["M"] += gu.T @ c["x"]
        gx = gx_prev + gu @ bk["M"]
    return gx + gh_in


def agent_weights(p, E, H, D):
    return dict(We=p["feat_embedding.weight"], be=p["feat_embedding.bias"],
                Wo=p["q_basic.weight"], bo=p["q_basic.bias"],
                blocks=derive(p, "transformer.", E, H, D))


def agent_unroll_with_grads(p, obs, h0, gq_all, gh_all, *, E, H, D, n, Fd):
    """Forward unroll + BPTT with external grads gq [b,T,A,nA], gh [b,T,A,E].
    Returns q, h, param grads (reference keys) and grads wrt h0."""
    W = agent_weights(p, E, H, D)
    b, T, A, _ = obs.shape
    R = b * A
    hs = [h0.reshape(R, E)]
    qs, cs = [], []
    for t in range(T):
        o = obs[:, t].reshape(R, n, Fd)
        q, hn, cc = agent_step_fwd(W, hs[-1], o, H)
        qs.append(q)
        hs.append(hn)
        cs.append(cc)
    g = dict(We=torch.zeros_like(W["We"]), be=torch.zeros_like(W["be"]),
             Wo=torch.zeros_like(W["Wo"]), bo=torch.zeros_like(W["bo"]),
             blocks=_zero_gblocks(W["blocks"]))
    gh = torch.zeros(R, E, dtype=h0.dtype)
    for t in reversed(range(T)):
        o = obs[:, t].reshape(R, n, Fd)
        gh = agent_step_bwd(W, hs[t], o, H, hs[t + 1], cs[t], gh + gh_all[:, t].reshape(R, E),
                            gq_all[:, t].reshape(R, -1), g)
    grads = fold_grads(p, "transformer.", E, H, D, g["blocks"])
    grads.update({"feat_embedding.weight": g["We"], "feat_embedding.bias": g["be"],
                  "q_basic.weight": g["Wo"], "q_basic.bias": g["bo"]})
    q = torch.stack(qs, 1).view(b, A, T, -1).transpose(1, 2)
    h = torch.stack(hs[1:], 1).view(b, A, T, E).transpose(1, 2)
    return q, h, grads, gh.view(b, A, E)


# ----------------------------------------------------------------------------- mixer
def mixer_step_fwd(W, qv, hid, hw, st, H):
    """One mixer step for b episodes. qv [b,A], hid [b,A,E], hw [b,3,E], st [b,ns,Fs]."""
    b, A, E = hid.shape
    emb = st @ W["We"].T + W["be"]
    X0 = torch.cat([emb, hid, hw], 1)                # [b,Lk,E]
    ns = st.shape[1]
    x = X0[:, ns:]                                   # [b,A+3,E] queries
    caches = []
    for bk in W["blocks"]:
        Rq = x.shape[1]
        u = (x @ bk["M"].T).view(b, Rq, H, E)
        s = torch.einsum("bqhe,bke->bqhk", u, X0)
        pr = torch.softmax(s, -1)
        z = torch.einsum("bqhk,bke->bqhe", pr, X0)
        a = z.reshape(b, Rq, H * E) @ bk["N"].T + bk["bu"]
        xf = x.reshape(b * Rq, E)
        xo, cc = _ffn_ln_fwd(bk, a.reshape(b * Rq, E), xf)
        cc.update(x=xf, u=u, pr=pr, z=z)
        caches.append(cc)
        x = xo.view(b, Rq, E)
    w1 = x[:, :A].abs()
    b1 = x[:, A]
    w2 = x[:, A + 1].abs()
    pre2 = x[:, A + 2] @ W["hb2w"][0] + W["hb2b"][0]
    b2 = torch.relu(pre2)
    pre_h = torch.einsum("ba,bae->be", qv, w1) + b1
    hidden = F.elu(pre_h)
    y = (hidden * w2).sum(-1) + b2
    cache = dict(X0=X0, caches=caches, out=x, pre_h=pre_h, hidden=hidden, pre2=pre2, st=st)
    return y, x[:, A:A + 3], cache


def mixer_step_bwd(W, qv, cache, gy, ghw_out, H, g):
    """Backward of one mixer step. Returns grads wrt qv [b,A], hid [b,A,E], hw [b,3,E]."""
    X0, out = cache["X0"], cache["out"]
    b, Rq, E = out.shape
    A = Rq - 3
    ns = X0.shape[1] - Rq
    gout = torch.zeros_like(out)
    gout[:, A:A + 3] += ghw_out
    w1 = out[:, :A].abs()
    w2 = out[:, A + 1].abs()
    hidden = cache["hidden"]
    # y = hidden.w2 + relu(pre2)
    gw2 = gy[:, None] * hidden
    ghid = gy[:, None] * w2
    gpre2 = gy * (cache["pre2"] > 0)
    g["hb2w"] += (gpre2[:, None] * out[:, A + 2]).sum(0)[None]
    g["hb2b"] += gpre2.sum()[None]
    gout[:, A + 2] += gpre2[:, None] * W["hb2w"][0]
    gout[:, A + 1] += gw2 * torch.sign(out[:, A + 1])
    pre_h = cache["pre_h"]
    gpre = ghid * torch.where(pre_h > 0, torch.ones_like(pre_h), torch.exp(pre_h))
    gout[:, A] += gpre
    gqv = torch.einsum("be,bae->ba", gpre, w1)
    gout[:, :A] += qv[..., None] * gpre[:, None, :] * torch.sign(out[:, :A])
    gX0 = torch.zeros_like(X0)
    gx = gout.reshape(b * Rq, E)
    for d in reversed(range(len(W["blocks"]))):
        bk, c, gb = W["blocks"][d], cache["caches"][d], g["blocks"][d]
        ga = _ffn_ln_bwd(bk, c, gx, gb)
        gx_prev = ga.clone()
        gb["N"] += ga.T @ c["z"].reshape(b * Rq, H * E)
        gb["bu"] += ga.sum(0)
        gz = (ga @ bk["N"]).view(b, Rq, H, E)
        pr, u = c["pr"], c["u"]
        gX0 += torch.einsum("bqhk,bqhe->bke", pr, gz)
        gp = torch.einsum("bqhe,bke->bqhk", gz, X0)
        gs = pr * (gp - (pr * gp).sum(-1, keepdim=True))
        gu = torch.einsum("bqhk,bke->bqhe", gs, X0)
        gX0 += torch.einsum("bqhk,bqhe->bke", gs, u)
        gu = gu.reshape(b * Rq, H * E)
        gb["M"] += gu.T @ c["x"]
        gx = gx_prev + gu @ bk["M"]
    gX0[:, ns:] += gx.view(b, Rq, E)
    gemb = gX0[:, :ns]
    g["We"] += torch.einsum("bje,bjf->ef", gemb, cache["st"])
    g["be"] += gemb.sum((0, 1))
    return gqv, gX0[:, ns:ns + A], gX0[:, ns + A:]


def mixer_weights(p, E, H, D):
    return dict(We=p["feat_embedding.weight"], be=p["feat_embedding.bias"],
                hb2w=p["hyper_b2.weight"], hb2b=p["hyper_b2.bias"],
                blocks=derive(p, "transformer.", E, H, D))


def mixer_unroll_with_grads(p, qvals, hidden, states, hw0, gy_all, ghw_all, *, E, H, D, Fs):
    W = mixer_weights(p, E, H, D)
    b, T, A = qvals.shape
    hws = [hw0]
    ys, cs = [], []
    for t in range(T):
        st = states[:, t].reshape(b, -1, Fs)
        y, hw, c = mixer_step_fwd(W, qvals[:, t], hidden[:, t], hws[-1], st, H)
        ys.append(y)
        hws.append(hw)
        cs.append(c)
    g = dict(We=torch.zeros_like(W["We"]), be=torch.zeros_like(W["be"]),
             hb2w=torch.zeros_like(W["hb2w"]), hb2b=torch.zeros_like(W["hb2b"]),
             blocks=_zero_gblocks(W["blocks"]))
    ghw = torch.zeros_like(hw0)
    gq = torch.zeros_like(qvals)
    ghid = torch.zeros_like(hidden)
    for t in reversed(range(T)):
        gqt, ght, ghw = mixer_step_bwd(W, qvals[:, t], cs[t], gy_all[:, t], ghw + ghw_all[:, t], H, g)
        gq[:, t] = gqt
        ghid[:, t] = ght
    grads = fold_grads(p, "transformer.", E, H, D, g["blocks"])
    grads.update({"feat_embedding.weight": g["We"], "feat_embedding.bias": g["be"],
                  "hyper_b2.weight": g["hb2w"], "hyper_b2.bias": g["hb2b"]})
    return torch.stack(ys, 1), torch.stack(hws[1:], 1), grads, gq, ghid, ghw
