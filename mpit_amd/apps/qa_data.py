"""QA data preparation for BiCNN (BiCNN/prepareData.lua:1-299).

File formats (tab separated, as read by the reference):
* embedding file: ``word<TAB>v1 v2 ... vD``
* train file:     ``labels<TAB>(ignored)<TAB>question words<TAB>answer words``
* valid / test:   ``labels<TAB>question words<TAB>pool of answer labels``
* label2answer:   ``label<TAB>answer words``

Sentences are padded with ``convWidth`` SENTBEGIN tokens in front and ``convWidth-1``
SENTEND tokens behind (prepareData.lua:90,102); out-of-vocabulary words get uniform
random embeddings. Index 0 is reserved for batch padding here (the reference had no
batching), so SENTBEGIN=1 and SENTEND=2 as in the reference.

:func:`synthetic_qa` builds a learnable stand-in with the same structure (the reference's
data files are not in the repository: .MISSING_LARGE_BLOBS).
"""
from __future__ import annotations

import random
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch

PAD, SENTBEGIN, SENTEND = 0, 1, 2


@dataclass
class QAData:
    word2idx: Dict[str, int] = field(default_factory=lambda: {"<pad>": PAD, "SENTBEGIN": SENTBEGIN, "SENTEND": SENTEND})
    vectors: List[List[float]] = field(default_factory=list)
    train: List[tuple] = field(default_factory=list)  # (labels, q_ids, a_ids)
    valid: List[tuple] = field(default_factory=list)  # (labels, q_ids, pool)
    tests: List[List[tuple]] = field(default_factory=list)
    answers: Dict[int, List[int]] = field(default_factory=dict)  # label -> token ids
    emb_dim: int = 100
    conv_width: int = 2

    def _id(self, w: str, rng: random.Random) -> int:
        i = self.word2idx.get(w)
        if i is None:
            i = len(self.word2idx)
            self.word2idx[w] = i
            self.vectors.append([rng.random() for _ in range(self.emb_dim)])
        return i

    def encode(self, words: List[str], rng: random.Random) -> List[int]:
        k = self.conv_width
        return [SENTBEGIN] * k + [self._id(w, rng) for w in words] + [SENTEND] * (k - 1)

    def embedding_matrix(self) -> torch.Tensor:
        v = torch.zeros(len(self.word2idx), self.emb_dim)
        base = len(self.word2idx) - len(self.vectors)
        if self.vectors:
            v[base:] = torch.tensor(self.vectors)
        return v


def pad_batch(seqs: List[List[int]], min_len: int = 2) -> torch.Tensor:
    T = max(min_len, max(len(s) for s in seqs))
    out = torch.full((len(seqs), T), PAD, dtype=torch.long)
    for i, s in enumerate(seqs):
        out[i, : len(s)] = torch.tensor(s, dtype=torch.long)
    return out


def load_files(embedding: str, train: str, label2answer: str, valid: Optional[str] = None, tests=(),
               emb_dim: int = 100, conv_width: int = 2, seed: int = 1) -> QAData:
    rng = random.Random(seed)
    d = QAData(emb_dim=emb_dim, conv_width=conv_width)
    with open(embedding) as f:
        for line in f:
            k, _, v = line.rstrip("\n").partition("\t")
            d.word2idx[k] = len(d.word2idx)
            d.vectors.append([float(x) for x in v.split()])
    with open(label2answer) as f:
        for line in f:
            lab, _, txt = line.rstrip("\n").partition("\t")
            d.answers[int(lab)] = d.encode(txt.split(), rng)
    with open(train) as f:
        for line in f:
            parts = line.rstrip("\n").split("\t")
            labels = [int(x) for x in parts[0].split()]
            d.train.append((labels, d.encode(parts[2].split(), rng), d.encode(parts[3].split(), rng)))

    def eval_file(p):
        out = []
        with open(p) as f:
            for line in f:
                parts = line.rstrip("\n").split("\t")
                out.append(([int(x) for x in parts[0].split()], d.encode(parts[1].split(), rng),
                            [int(x) for x in parts[2].split()]))
        return out

    if valid:
        d.valid = eval_file(valid)
    d.tests = [eval_file(t) for t in tests]
    return d


def save_binary(d: QAData, path: str) -> None:
    """Prepared-data cache (the reference's ``-preloadBinary`` files written from
    prepareData.lua's tables, BiCNN/plaunch.lua:218-229): one file of plain containers +
    one tensor, loadable with ``torch.load(weights_only=True)`` (nothing executes)."""
    torch.save({
        "version": 1, "emb_dim": d.emb_dim, "conv_width": d.conv_width,
        "words": list(d.word2idx.keys()), "ids": list(d.word2idx.values()),
        "vectors": torch.tensor(d.vectors, dtype=torch.float32) if d.vectors else torch.zeros(0, d.emb_dim),
        "train": [[list(l), list(q), list(a)] for l, q, a in d.train],
        "valid": [[list(l), list(q), list(p)] for l, q, p in d.valid],
        "tests": [[[list(l), list(q), list(p)] for l, q, p in t] for t in d.tests],
        "answer_labels": list(d.answers.keys()), "answer_ids": list(d.answers.values()),
    }, path)


def load_binary(path: str) -> QAData:
    s = torch.load(path, weights_only=True)
    d = QAData(emb_dim=int(s["emb_dim"]), conv_width=int(s["conv_width"]))
    d.word2idx = dict(zip(s["words"], s["ids"]))
    d.vectors = s["vectors"].tolist()
    d.train = [tuple(x) for x in s["train"]]
    d.valid = [tuple(x) for x in s["valid"]]
    d.tests = [[tuple(x) for x in t] for t in s["tests"]]
    d.answers = dict(zip(s["answer_labels"], s["answer_ids"]))
    return d


T7_VOCAB = ("binary_mapWordStr2WordIdx", "binary_mapWordIdx2WordStr")


def load_t7_vocab(directory: str) -> Dict[str, int]:
    """The reference's shipped vocabulary caches (BiCNN/binary_mapWordStr2WordIdx and
    binary_mapWordIdx2WordStr, Torch7 tables written by prepareData.lua and loaded by
    plaunch.lua:222-223) through the plain-data Torch7 reader (mpit_amd/utils/t7.py: no
    torch object or function is ever constructed). The two maps must be mutually inverse
    over ids 1..n with SENTBEGIN = 1 and SENTEND = 2 (prepareData.lua:37-42); returns
    word -> id (the reference's 1-based ids, which are this package's ids too: 0 = pad)."""
    import os

    from ..utils import t7

    s2i = t7.load(os.path.join(directory, T7_VOCAB[0]))
    i2s = t7.load(os.path.join(directory, T7_VOCAB[1]))
    if not isinstance(s2i, dict) or not isinstance(i2s, dict):
        raise ValueError("t7 vocabulary: the caches must hold tables")
    n = len(s2i)
    if len(i2s) != n or sorted(i2s) != list(range(1, n + 1)):
        raise ValueError(f"t7 vocabulary: id map is not 1..{n}")
    for w, i in s2i.items():
        if i2s.get(i) != w:
            raise ValueError(f"t7 vocabulary: maps disagree on {w!r} -> {i}")
    if s2i.get("SENTBEGIN") != SENTBEGIN or s2i.get("SENTEND") != SENTEND:
        raise ValueError("t7 vocabulary: SENTBEGIN / SENTEND are not ids 1 / 2")
    return dict(sorted(s2i.items(), key=lambda kv: kv[1]))


def qa_from_vocab(word2idx: Dict[str, int], emb_dim: int = 100, conv_width: int = 2, seed: int = 1,
                  **synthetic) -> QAData:
    """QA data over a given vocabulary (ids as given, 0 = pad): embeddings uniform random as
    the reference's out-of-vocabulary words (prepareData.lua:95-97; the word-vector cache
    binary_mapWordIdx2Vector holds torch tensors and is not shipped), questions and answers
    drawn as in :func:`synthetic_qa` from the vocabulary's words."""
    rng = random.Random(seed)
    d = QAData(emb_dim=emb_dim, conv_width=conv_width)
    d.word2idx = {"<pad>": PAD}
    d.word2idx.update(word2idx)
    if sorted(d.word2idx.values()) != list(range(len(d.word2idx))):
        raise ValueError("qa_from_vocab: ids must be 0..n")
    d.vectors = [[rng.random() for _ in range(emb_dim)] for _ in range(len(d.word2idx) - 3)]
    words = [w for w in d.word2idx if w not in ("<pad>", "SENTBEGIN", "SENTEND")]
    return synthetic_qa(emb_dim=emb_dim, conv_width=conv_width, seed=seed, base=d, words=words, **synthetic)


def synthetic_qa(n_answers: int = 200, n_train: int = 2000, n_valid: int = 200, vocab: int = 2000, pool: int = 20,
                 emb_dim: int = 100, conv_width: int = 2, seed: int = 1, n_tests: int = 2,
                 base: Optional[QAData] = None, words: Optional[List[str]] = None) -> QAData:
    """Answers are random word sequences; a question shares 3 "key" words with its answer
    plus noise words, so GESD ranking is learnable. base / words: start from a given
    vocabulary and draw from its words (:func:`qa_from_vocab`)."""
    rng = random.Random(seed)
    d = base if base is not None else QAData(emb_dim=emb_dim, conv_width=conv_width)
    words = words if words is not None else [f"w{i}" for i in range(vocab)]
    for lab in range(n_answers):
        d.answers[lab] = d.encode(rng.sample(words, rng.randint(6, 12)), rng)
    ans_words = {lab: [w for w in d.answers[lab][conv_width:-(conv_width - 1) or None]] for lab in d.answers}
    idx2w = {i: w for w, i in d.word2idx.items()}

    def question(lab):
        keys = [idx2w[i] for i in rng.sample(ans_words[lab], 3)]
        return keys + rng.sample(words, rng.randint(2, 6))

    for _ in range(n_train):
        lab = rng.randrange(n_answers)
        d.train.append(([lab], d.encode(question(lab), rng), d.answers[lab]))
    def eval_set():
        out = []
        for _ in range(n_valid):
            lab = rng.randrange(n_answers)
            cands = list({lab} | set(rng.sample(range(n_answers), pool - 1)))
            out.append(([lab], d.encode(question(lab), rng), cands))
        return out

    d.valid = eval_set()
    d.tests = [eval_set() for _ in range(n_tests)]  # stand-ins for test1 / test2
    return d
