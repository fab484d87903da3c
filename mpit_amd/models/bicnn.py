"""BiCNN / GESD question-answer model (BiCNN/bicnn.lua:30-121), custom layers
(BiCNN/Normalize.lua, BiCNN/DivideConstant.lua) and the margin ranking objective.

Tower (weights shared by the Q, Q2, A+ and A- towers, ``:set()`` tying in the reference):
Embedding(V, 100) -> Linear(100, 200) -> Tanh -> Conv1d(200, 3000, k=2) -> max over time
-> ReLU -> L2 normalise. GESD similarity: ``1/(1+||a-b||) * 1/(1+exp(-(a.b+1)))``.
``mmode`` 1 compares Q with both answers; 2 uses a second question encoding for the
negative (BiCNN/bicnn.lua:87-116 — with tied weights the two are identical functions of
the same question, kept for parity).

MI355X adaptation: the reference runs one (question, answer) pair at a time; here a batch
of padded sequences is encoded at once (max-over-time masks the padding). Negative
sampling keeps the reference's semantics — per example, the first margin-violating draw
within ``maxnegsample`` (:func:`first_violations`, BiCNN/bicnn.lua:321-374) — with the
draws encoded in batched windows; :func:`margin_ranking_loss` is the cheaper
hardest-of-k alternative.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import register


class Normalize(nn.Module):
    """Lp normalisation over the last dim (BiCNN/Normalize.lua:1-86; autograd supplies
    the analytic Jacobian the reference wrote by hand)."""

    def __init__(self, p: float = 2.0, eps: float = 1e-10):
        super().__init__()
        self.p, self.eps = p, eps

    def forward(self, x):
        return x / x.norm(p=self.p, dim=-1, keepdim=True).clamp_min(self.eps)


class DivideConstant(nn.Module):
    """``y = c / x``, ``dx = -c g / x^2`` (BiCNN/DivideConstant.lua:4-25)."""

    def __init__(self, c: float = 1.0):
        super().__init__()
        self.c = c

    def forward(self, x):
        return self.c / x


def gesd(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """GESD similarity of row pairs (BiCNN/bicnn.lua:99-105)."""
    l2 = (a - b).norm(dim=-1)
    dot = (a * b).sum(-1)
    return (1.0 / (1.0 + l2)) * (1.0 / (1.0 + torch.exp(-(dot + 1.0))))


class BiCNN(nn.Module):
    def __init__(self, vocab: int = 22354, emb_dim: int = 100, hidden: int = 200, filters: int = 3000,
                 conv_width: int = 2, mmode: int = 1, pad_idx: int = 0):
        super().__init__()
        self.embed = nn.Embedding(vocab, emb_dim, padding_idx=pad_idx)
        self.hidden = nn.Linear(emb_dim, hidden)
        self.conv = nn.Conv1d(hidden, filters, conv_width)
        self.norm = Normalize(2)
        self.mmode = mmode
        self.pad_idx = pad_idx

    def encode(self, tok: torch.Tensor) -> torch.Tensor:
        """tok: [B, T] word ids (pad_idx = padding) -> [B, filters] unit embeddings."""
        h = torch.tanh(self.hidden(self.embed(tok)))  # [B, T, H]
        c = self.conv(h.transpose(1, 2))  # [B, F, T-k+1]
        k = self.conv.kernel_size[0]
        valid = (tok != self.pad_idx)
        # a window is valid when its LAST token is not padding (sentences are left-aligned,
        # so every token of the window is then a real one): exactly the windows of the
        # unpadded sentence
        vw = valid[:, k - 1:].unsqueeze(1)
        c = c.masked_fill(~vw, float("-inf"))
        m = c.max(dim=-1).values
        m = torch.nan_to_num(m, neginf=0.0)
        return self.norm(F.relu(m))

    def forward(self, q, a_pos, a_neg):
        eq = self.encode(q)
        ep = self.encode(a_pos)
        b, nneg, t = a_neg.shape
        en = self.encode(a_neg.reshape(b * nneg, t)).reshape(b, nneg, -1)
        eq2 = eq if self.mmode == 1 else self.encode(q)
        s_pos = gesd(eq, ep)
        s_neg = gesd(eq2.unsqueeze(1).expand_as(en), en)  # [B, nneg]
        return s_pos, s_neg


def margin_ranking_loss(s_pos, s_neg, margin: float = 0.009):
    """nn.MarginRankingCriterion(margin) with the hardest sampled negative
    (BiCNN/bicnn.lua:121, :279-420)."""
    hard = s_neg.max(dim=-1).values
    return F.relu(margin - s_pos + hard).mean()


def draw_negatives(rng, n_answers: int, positives, maxneg: int) -> list:
    """The reference's per-example draw sequence: uniform labels with the example's
    positives rejected, ``maxneg`` draws (BiCNN/bicnn.lua:322-333; labels are 0-based
    here). Drawn up front so the scan below can batch the encodes."""
    pos = set(positives)
    if len(pos) >= n_answers:
        return []
    out = []
    while len(out) < maxneg:
        x = rng.randrange(n_answers)
        if x not in pos:
            out.append(x)
    return out


@torch.no_grad()
def first_violations(model: "BiCNN", eq: torch.Tensor, s_pos: torch.Tensor, draws: list, answers,
                     margin: float, pad_fn, chunk: int = 8) -> list:
    """Parity negative sampling (BiCNN/bicnn.lua:321-374): for every example ``i`` scan its
    draw sequence ``draws[i]`` in order and return the first negative label whose
    similarity violates the margin (``s_pos - s_neg < margin``), or ``None`` when all
    ``maxnegsample`` draws satisfy it (the reference then skips the example: ``goto
    continue``).

    The reference encodes one negative at a time; here the next draws of every
    still-unresolved example are encoded in one batched pass (unique labels only, the
    window doubling from ``chunk`` each round), so the scan costs O(log maxnegsample)
    batched encodes instead of one tiny encode per draw. The selected label is the
    sequential scan's: the first violating draw in draw order.
    """
    b = eq.shape[0]
    chosen = [None] * b
    live = [i for i in range(b) if draws[i]]
    start, width = 0, chunk
    maxlen = max((len(d) for d in draws), default=0)
    dev = eq.device
    while live and start < maxlen:
        seqs = [draws[i][start: start + width] for i in live]
        labs = sorted({x for s in seqs for x in s})
        if not labs:
            break
        emb = model.encode(pad_fn([answers[x] for x in labs]).to(dev))
        row = {x: j for j, x in enumerate(labs)}
        w = max(len(s) for s in seqs)
        idx = torch.tensor([[row[x] for x in s] + [0] * (w - len(s)) for s in seqs], device=dev)
        valid = torch.tensor([[1] * len(s) + [0] * (w - len(s)) for s in seqs], device=dev, dtype=torch.bool)
        li = torch.tensor(live, device=dev)
        sn = gesd(eq[li].unsqueeze(1).expand(-1, w, -1), emb[idx])  # [n_live, w]
        viol = ((s_pos[li].unsqueeze(1) - sn) < margin) & valid
        has = viol.any(1).tolist()
        first = viol.to(torch.int32).argmax(1).tolist()
        nxt = []
        for k, i in enumerate(live):
            if has[k]:
                chosen[i] = seqs[k][first[k]]
            else:
                nxt.append(i)
        live = nxt
        start += width
        width *= 2
    return chosen


def parity_loss(model: "BiCNN", q, a_pos, a_neg, margin: float):
    """Summed MarginRankingCriterion over the selected (violating) examples — the
    reference accumulates ``f = f + currErr`` and the gradients of every example of the
    batch without averaging (BiCNN/bicnn.lua:376-397)."""
    sp, sn = model(q, a_pos, a_neg.unsqueeze(1))
    return F.relu(margin - sp + sn[:, 0]).sum()


def per_example_grads(model: "BiCNN", flat, q, a_pos, a_neg, margin: float) -> torch.Tensor:
    """[n, flat.numel] fp32: row k = the gradient of example k's margin loss alone, laid out
    like the flat parameter vector (``flat``: utils/flat.py FlatParams of ``model``). One
    batched backward (torch.func.vmap over per-example grads) instead of the reference's
    one backward per example."""
    from torch.func import functional_call, grad, vmap

    names = [n for n, _ in model.named_parameters()]
    params = {n: p.detach() for n, p in model.named_parameters()}

    def one(pr, qi, api, ani):
        sp, sn = functional_call(model, pr, (qi[None], api[None], ani[None, None]))
        return F.relu(margin - sp + sn[:, 0]).sum()

    gd = vmap(grad(one), in_dims=(None, 0, 0, 0))(params, q, a_pos, a_neg)
    n = q.shape[0]
    out = torch.zeros((n, flat.numel), dtype=torch.float32, device=q.device)
    for name, p, off in zip(names, flat.params, flat.offsets):
        g = gd[name]
        if flat.channels_last and p.dim() == 4:
            g = g.permute(0, 1, 3, 4, 2)  # [n, o, h, w, i]: the flat buffer's NHWC order
        out[:, off: off + p.numel()] = g.reshape(n, -1)
    return out


def parity_grad_(model: "BiCNN", flat, q, a_pos, a_neg, margin: float, l1: float, l2: float, clip: float,
                 chunk: int = 16) -> torch.Tensor:
    """The reference's per-example gradient rule for the violating examples (in order):
    ``G += g_k; G += l1*sign(p) + l2*p; G = clamp(G, -clip, clip)`` after EVERY example
    (BiCNN/bicnn.lua:376-409; ``clip <= 0`` = no clamp). Writes G into ``flat.grad`` and
    returns the summed loss ``Σ_k (err_k + l1*|p|_1 + l2*|p|^2/2)`` (``f`` of the feval).
    Per-example gradients come ``chunk`` examples at a time (:func:`per_example_grads`);
    the regularise + clamp chain runs as ONE fused pass per chunk (ops.clamp_scan_)."""
    from .. import ops

    G = flat.grad
    G.zero_()
    n = q.shape[0]
    for s in range(0, n, chunk):
        g = per_example_grads(model, flat, q[s:s + chunk], a_pos[s:s + chunk], a_neg[s:s + chunk], margin)
        ops.clamp_scan_(G, g, flat.flat[: flat.numel], l1, l2, clip)
    with torch.no_grad():
        loss = parity_loss(model, q, a_pos, a_neg, margin)
        if l1 or l2:
            nm = ops.norms(flat.flat[: flat.numel])
            loss = loss + n * (l1 * nm[0] + 0.5 * l2 * nm[1])
    return loss


@register("bicnn")
def bicnn(num_classes=None, **kw):
    return BiCNN(**kw)
