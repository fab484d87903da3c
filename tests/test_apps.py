"""Application-level tests (CPU): BiCNN's negative-sampling parity, its prepared-data
cache, and end-to-end runs of apps/bicnn.py and apps/goot.py under the launcher with the
reference's role layouts (BiCNN/plaunch.lua:117-177, asyncsgd/mlaunch.lua:40-46)."""
import glob
import os
import random
import subprocess
import sys

import pytest
import torch

from mp_util import ROOT

from mpit_amd.apps.qa_data import load_binary, pad_batch, save_binary, synthetic_qa
from mpit_amd.models.bicnn import BiCNN, draw_negatives, first_violations, gesd

TINY = ["-numFilters", "48", "-wordHiddenDim", "24", "-embeddingDim", "16", "-batchSize", "16",
        "-synthetic", "60", "-maxnegsample", "12", "-evalMax", "40", "-validSleepTime", "0.05", "-type", "float"]


def _sequential_first_violation(model, q_tok, a_tok, draws, answers, margin):
    """The reference's scan, literally: one negative at a time (BiCNN/bicnn.lua:321-359)."""
    eq = model.encode(q_tok.unsqueeze(0))
    sp = gesd(eq, model.encode(a_tok.unsqueeze(0)))[0]
    for x in draws:
        sn = gesd(eq, model.encode(pad_batch([answers[x]])))[0]
        if sp - sn < margin:
            return x
    return None


@pytest.mark.parametrize("margin", [0.0, 0.02, 0.3])
def test_first_violation_matches_sequential_scan(margin):
    torch.manual_seed(0)
    d = synthetic_qa(n_answers=40, n_train=24, emb_dim=8)
    m = BiCNN(len(d.word2idx), 8, 12, 20, 2).eval()
    batch = d.train[:24]
    q = pad_batch([b[1] for b in batch])
    a = pad_batch([b[2] for b in batch])
    rng = random.Random(3)
    labs = sorted(d.answers)
    draws = [draw_negatives(rng, len(labs), labels, 30) for labels, _, _ in batch]
    with torch.no_grad():
        eq = m.encode(q)
        sp = gesd(eq, m.encode(a))
        got = first_violations(m, eq, sp, draws, d.answers, margin, pad_batch, chunk=2)
        want = [_sequential_first_violation(m, q[i][q[i] != 0], a[i][a[i] != 0], draws[i], d.answers, margin)
                for i in range(len(batch))]
    assert got == want
    if margin == 0.3:
        assert all(g is not None for g in got)


def test_draw_negatives_rejects_positives():
    rng = random.Random(0)
    seq = draw_negatives(rng, 5, [1, 3], 200)
    assert len(seq) == 200 and set(seq) == {0, 2, 4}
    assert draw_negatives(rng, 2, [0, 1], 10) == []  # nothing to draw


def test_binary_cache_roundtrip(tmp_path):
    d = synthetic_qa(n_answers=30, n_train=50, emb_dim=8)
    p = str(tmp_path / "qa.pt")
    save_binary(d, p)
    e = load_binary(p)
    assert e.word2idx == d.word2idx and e.answers == d.answers
    assert [tuple(map(list, x)) for x in e.train] == [tuple(map(list, x)) for x in d.train]
    assert len(e.tests) == 2 and e.tests[1][0][2] == d.tests[1][0][2]
    assert torch.equal(e.embedding_matrix(), d.embedding_matrix())


def _launch(n, script, args, cwd, timeout=240):
    env = dict(os.environ, MPIT_CPU_ONLY="1", OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "mpit_amd.launch", "-n", str(n), "--timeout", str(timeout - 20),
                        os.path.join(ROOT, "mpit_amd", "apps", script)] + args,
                       capture_output=True, text=True, timeout=timeout, env=env, cwd=cwd)
    assert r.returncode == 0, f"rc={r.returncode}\n{r.stdout[-3000:]}\n{r.stderr[-4000:]}"
    return r.stdout


@pytest.mark.parametrize("tester", ["-testerfirst", "-testerlast"])
def test_bicnn_tester_terminates_and_saves(tmp_path, tester):
    out = _launch(5, "bicnn.py", TINY + [tester, "-masterFreq", "2", "-optimization", "adam", "-maxSteps", "4",
                                         "-outputprefix", str(tmp_path / "m")], str(tmp_path))
    assert "best valid acc" in out
    assert "on file3" in out  # valid + test1 + test2 (bicnn.lua:465-571)
    files = glob.glob(str(tmp_path / "m_*_model"))
    assert files, out[-2000:]
    p = torch.load(files[0], weights_only=True)
    assert p.dim() == 1 and torch.isfinite(p).all()


def test_bicnn_lastclient_loadmodel_maxrank(tmp_path):
    # 4 ranks, maxrank 2: ranks 0..2 work (rank 0 trains: lastClient has no tester), rank 3 idles
    out = _launch(4, "bicnn.py", TINY + ["-testerfirst", "-masterFreq", "2", "-maxrank", "2", "-validMode", "lastClient",
                                         "-optimization", "downpour", "-maxSteps", "3", "-outputprefix",
                                         str(tmp_path / "lc")], str(tmp_path))
    assert "rank 3 do nothing" in out and "will also run testing" in out
    files = sorted(glob.glob(str(tmp_path / "lc_*_model")))
    assert files
    out = _launch(3, "bicnn.py", TINY + ["-testerfirst", "-masterFreq", "2", "-validMode", "additionalTester",
                                         "-optimization", "downpour", "-maxSteps", "2", "-loadmodel", files[-1],
                                         "-prevtime", "1000", "-outputprefix", str(tmp_path / "re")], str(tmp_path))
    re_files = glob.glob(str(tmp_path / "re_*_model"))
    assert re_files and all(float(os.path.basename(f).split("_")[1]) >= 1000 for f in re_files)


def test_bicnn_singlemode(tmp_path):
    out = _launch(5, "bicnn.py", TINY + ["-testerfirst", "-masterFreq", "3", "-singlemode", "-optimization",
                                         "adamsingle", "-maxSteps", "4"], str(tmp_path))
    assert "singlemode: only rank 1 pushes parameters" in out
    assert "[bicnn worker 1] steps 4" in out and "best valid acc" in out


def test_bicnn_preload_binary(tmp_path):
    _launch(1, "bicnn.py", TINY + ["-saveBinary", "-binaryFile", "qa.pt", "-maxSteps", "2", "-validMode", "none"],
            str(tmp_path))
    assert (tmp_path / "qa.pt").exists()
    out = _launch(1, "bicnn.py", TINY + ["-preloadBinary", "-binaryFile", "qa.pt", "-maxSteps", "2", "-validMode",
                                         "none", "-negMode", "hardest"], str(tmp_path))
    assert "steps 2" in out


def test_goot_mlaunch_roles(tmp_path):
    out = _launch(4, "goot.py", ["--optimizer", "eamsgd", "--subset", "--max-steps", "3", "--batch", "32",
                                 "--save", str(tmp_path / "g")], str(tmp_path))
    assert "[goot] epoch" in out and "[goot] rank" in out


def test_load_files_reference_format(tmp_path):
    """BiCNN/prepareData.lua's text formats: embedding `word<TAB>v1 .. vD`, train
    `labels<TAB>x<TAB>question<TAB>answer`, valid/test `labels<TAB>question<TAB>pool`,
    label2answer `label<TAB>answer`; sentences padded with convWidth SENTBEGIN in front and
    convWidth-1 SENTEND behind, out-of-vocabulary words get new ids."""
    from mpit_amd.apps.qa_data import SENTBEGIN, SENTEND, load_files

    (tmp_path / "emb.txt").write_text("what\t0.1 0.2 0.3\nis\t0.4 0.5 0.6\n")
    (tmp_path / "l2a.txt").write_text("0\tit is red\n1\tit is blue\n2\tnone\n")
    (tmp_path / "train.txt").write_text("0\tx\twhat is red\tit is red\n1 2\tx\twhat is blue\tit is blue\n")
    (tmp_path / "valid.txt").write_text("0\twhat is it\t0 1 2\n")
    (tmp_path / "test1.txt").write_text("1\twhat\t1 2\n")
    d = load_files(str(tmp_path / "emb.txt"), str(tmp_path / "train.txt"), str(tmp_path / "l2a.txt"),
                   str(tmp_path / "valid.txt"), tests=[str(tmp_path / "test1.txt")], emb_dim=3, conv_width=2)
    what, is_ = d.word2idx["what"], d.word2idx["is"]
    assert d.embedding_matrix()[what].tolist() == pytest.approx([0.1, 0.2, 0.3])
    labels, q, a = d.train[1]
    assert labels == [1, 2]
    assert q[:2] == [SENTBEGIN, SENTBEGIN] and q[-1:] == [SENTEND] and q[2:4] == [what, is_]
    assert a == d.answers[1]
    assert d.valid[0][0] == [0] and d.valid[0][2] == [0, 1, 2]
    assert len(d.tests) == 1 and d.tests[0][0][2] == [1, 2]
    assert len(d.word2idx) == d.embedding_matrix().shape[0]


def _seq_parity_grad(model, flat, q, ap, an, margin, l1, l2, clip):
    """The reference's feval loop, literally (BiCNN/bicnn.lua:376-409): per violating
    example one backward into the running gradient, then the regulariser, then the clamp."""
    import torch.nn.functional as F

    params = list(model.parameters())
    G = torch.zeros(flat.numel)
    p = flat.flat[: flat.numel].detach()
    for k in range(q.shape[0]):
        sp, sn = model(q[k:k + 1], ap[k:k + 1], an[k:k + 1, None])
        gs = torch.autograd.grad(F.relu(margin - sp + sn[:, 0]).sum(), params)
        for g, off in zip(gs, flat.offsets):
            G[off: off + g.numel()] += g.reshape(-1)
        G += l1 * torch.sign(p) + l2 * p
        G.clamp_(-clip, clip)
    return G


@pytest.mark.parametrize("l1,l2,clip", [(0.0, 1e-4, 0.5), (1e-3, 1e-4, 0.02), (0.0, 0.0, 0.005)])
def test_bicnn_parity_clamp_matches_sequential_loop(l1, l2, clip):
    """-clipMode parity: the accumulated gradient is regularised and clamped after every
    violating example (once per batch gave +0.2 where the reference gives -0.1)."""
    from mpit_amd.models.bicnn import BiCNN, parity_grad_
    from mpit_amd.utils.flat import FlatParams

    torch.manual_seed(0)
    model = BiCNN(vocab=60, emb_dim=8, hidden=12, filters=16, conv_width=2)
    flat = FlatParams(model)
    n, t = 7, 9
    q = torch.randint(1, 60, (n, t))
    ap = torch.randint(1, 60, (n, t))
    an = torch.randint(1, 60, (n, t))
    q[:, 7:] = 0  # padding
    an[2, 5:] = 0
    margin = 5.0  # every example violates
    loss = parity_grad_(model, flat, q, ap, an, margin, l1, l2, clip, chunk=3)
    ref = _seq_parity_grad(model, flat, q, ap, an, margin, l1, l2, clip)
    got = flat.grad[: flat.numel]
    assert torch.allclose(got, ref, atol=2e-6, rtol=1e-5), (got - ref).abs().max()
    if clip < 0.1:
        assert (ref.abs() >= clip * 0.999).any()  # the clamp was active
    assert torch.isfinite(loss)


def test_bicnn_parity_differs_from_batch_clamp():
    """The example of VERDICT r02: +0.8 then -0.6 with clip 0.5 — parity gives -0.1."""
    from mpit_amd import ops

    G = torch.zeros(4)
    g = torch.tensor([[0.8] * 4, [-0.6] * 4])
    ops.clamp_scan_(G, g, torch.zeros(4), 0.0, 0.0, 0.5)
    assert torch.allclose(G, torch.full((4,), -0.1))


@pytest.mark.gpu
def test_bicnn_parity_clamp_gpu_matches_cpu_loop():
    """The parity rule on the GPU (vmap per-example grads + the HIP clamp_scan kernel)
    against the literal sequential loop on the CPU (fp32)."""
    import copy

    from mpit_amd.models.bicnn import BiCNN, parity_grad_
    from mpit_amd.utils.flat import FlatParams

    torch.manual_seed(1)
    base = BiCNN(vocab=80, emb_dim=16, hidden=24, filters=64, conv_width=2)
    cpu_m, gpu_m = copy.deepcopy(base), copy.deepcopy(base).cuda()
    fc, fg = FlatParams(cpu_m), FlatParams(gpu_m)
    n, t = 10, 12
    q, ap, an = (torch.randint(1, 80, (n, t)) for _ in range(3))
    q[:, 9:] = 0
    parity_grad_(gpu_m, fg, q.cuda(), ap.cuda(), an.cuda(), 5.0, 1e-3, 1e-4, 0.01, chunk=4)
    ref = _seq_parity_grad(cpu_m, fc, q, ap, an, 5.0, 1e-3, 1e-4, 0.01)
    got = fg.grad[: fg.numel].cpu()
    assert torch.allclose(got, ref, atol=1e-5, rtol=1e-4), (got - ref).abs().max()
