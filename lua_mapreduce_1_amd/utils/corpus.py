"""Synthetic corpora shaped like the reference's headline workload.

The reference benchmarks word-count on Europarl-v7 English: 1,965,734 lines,
49,158,635 whitespace tokens, split into 197 files of at most 10,000 lines
(/root/reference/README.md:43-46, examples/WordCountBig/taskfn.lua:6-11).
There is no network here, so :func:`europarl_like` generates a corpus with the
same line/token/split counts, a Zipf-Mandelbrot vocabulary and English-like
word lengths (≈5.9 bytes per token incl. separator, ≈290 MB), deterministically
from a seed.
"""
from __future__ import annotations

import os

import numpy as np

EUROPARL_LINES = 1_965_734
EUROPARL_WORDS = 49_158_635
EUROPARL_SPLIT_LINES = 10_000


def make_vocab(size: int, rng: np.random.Generator, long_frac: float = 0.002) -> list[bytes]:
    """Unique byte-string vocabulary; frequent (low-rank) words are short."""
    letters = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz", dtype=np.uint8)
    ranks = np.arange(size, dtype=np.float64)
    mean_len = 1.1 + 0.62 * np.log1p(ranks)
    lens = np.clip(np.round(mean_len + rng.normal(0, 1.0, size)), 1, 24).astype(np.int64)
    nlong = int(size * long_frac)
    if nlong:
        idx = rng.choice(np.arange(size // 4, size), nlong, replace=False)
        lens[idx] = rng.integers(25, 90, nlong)
    seen: set[bytes] = set()
    out: list[bytes] = []
    punct = [b",", b".", b"?", b":", b";"]
    for r, n in enumerate(lens):
        while True:
            w = letters[rng.integers(0, 26, int(n))].tobytes()
            if r % 7 == 3:
                w = w[:1].upper() + w[1:]
            if r % 11 == 5 and n > 2:
                w = w[:-1] + punct[r % len(punct)]
            if w not in seen:
                seen.add(w)
                out.append(w)
                break
            n = n + 1 if rng.random() < 0.3 else n
    return out


def zipf_probs(size: int, s: float = 1.05, q: float = 2.7) -> np.ndarray:
    p = 1.0 / np.power(np.arange(size, dtype=np.float64) + q, s)
    return p / p.sum()


def europarl_like(seed: int = 1234, lines: int = EUROPARL_LINES, words: int = EUROPARL_WORDS,
                  split_lines: int = EUROPARL_SPLIT_LINES, vocab_size: int = 300_000, return_counts: bool = False,
                  return_bigrams: bool = False):
    """List of split byte strings (each ends with a newline); with
    ``return_counts`` also the vocabulary and every word's exact number of
    occurrences (the per-key ground truth of a word count); with
    ``return_bigrams`` (implies the vocabulary) also the distinct bigrams of
    the corpus as sorted codes ``first * vocab_size + second`` (word ids of
    two consecutive tokens of one line) and their counts."""
    return_counts = return_counts or return_bigrams
    bigram_codes = []
    rng = np.random.default_rng(seed)
    vocab = make_vocab(vocab_size, rng)
    vlen = np.array([len(w) for w in vocab], dtype=np.int64)
    voff = np.zeros(vocab_size + 1, dtype=np.int64)
    np.cumsum(vlen, out=voff[1:])
    vbytes = np.frombuffer(b"".join(vocab), dtype=np.uint8)
    cdf = np.cumsum(zipf_probs(vocab_size))
    cdf[-1] = 1.0
    # words per line: gamma-distributed around the Europarl mean, >= 1
    mean = words / lines
    wpl = np.maximum(1, np.round(rng.gamma(2.2, mean / 2.2, lines))).astype(np.int64)
    diff = int(words - wpl.sum())
    while diff != 0:
        idx = rng.integers(0, lines, min(abs(diff), lines))
        if diff > 0:
            np.add.at(wpl, idx, 1)
        else:
            ok = wpl[idx] > 1
            np.add.at(wpl, idx[ok], -1)
        diff = int(words - wpl.sum())
    splits = []
    counts = np.zeros(vocab_size, dtype=np.int64)
    for s0 in range(0, lines, split_lines):
        lw = wpl[s0:s0 + split_lines]
        nt = int(lw.sum())
        tok = np.searchsorted(cdf, rng.random(nt), side="right")
        tok = np.minimum(tok, vocab_size - 1)
        if return_counts:
            counts += np.bincount(tok, minlength=vocab_size)
        if return_bigrams and nt > 1:
            same_line = np.ones(nt - 1, bool)
            same_line[np.cumsum(lw)[:-1] - 1] = False  # token i is the last of its line
            c = tok[:-1] * np.int64(vocab_size) + tok[1:]
            bigram_codes.append(c[same_line])
        tl = vlen[tok]
        # separator after each token: space, or newline at end of line
        sep = np.full(nt, ord(" "), dtype=np.uint8)
        sep[np.cumsum(lw) - 1] = ord("\n")
        start = np.zeros(nt + 1, dtype=np.int64)
        np.cumsum(tl + 1, out=start[1:])
        total = int(start[-1])
        ti = np.repeat(np.arange(nt), tl + 1)
        ci = np.arange(total, dtype=np.int64) - start[ti]
        isw = ci < tl[ti]
        buf = np.empty(total, dtype=np.uint8)
        buf[isw] = vbytes[voff[tok[ti[isw]]] + ci[isw]]
        buf[~isw] = sep
        splits.append(buf.tobytes())
    if return_bigrams:
        codes, ccount = np.unique(np.concatenate(bigram_codes) if bigram_codes else np.zeros(0, np.int64),
                                  return_counts=True)
        return splits, vocab, counts, (codes, ccount)
    if return_counts:
        return splits, vocab, counts
    return splits


def write_splits(splits: list[bytes], directory: str, prefix: str = "split") -> list[str]:
    os.makedirs(directory, exist_ok=True)
    paths = []
    for i, s in enumerate(splits):
        p = os.path.join(directory, f"{prefix}{i:05d}.txt")
        with open(p, "wb") as f:
            f.write(s)
        paths.append(p)
    return paths


def tricky_text(rng: np.random.Generator, nbytes: int) -> bytes:
    """Adversarial bytes for tokenizer tests: all whitespace kinds, NULs, high
    bytes, long tokens crossing 4 KiB tiles / 64 KiB chunks, whitespace runs."""
    ws = b" \t\n\v\f\r"
    out = bytearray()
    while len(out) < nbytes:
        r = rng.random()
        if r < 0.55:
            n = int(rng.integers(1, 12))
            out += bytes(rng.integers(33, 127, n).astype(np.uint8))
        elif r < 0.6:
            n = int(rng.integers(13, 40))
            out += bytes(rng.integers(33, 127, n).astype(np.uint8))
        elif r < 0.605:
            n = int(rng.integers(60, 9000))
            out += bytes(rng.integers(33, 127, n).astype(np.uint8))
        elif r < 0.62:
            n = int(rng.integers(1, 20))
            b = rng.integers(0, 256, n).astype(np.uint8)
            b = np.array([x if x not in ws else 0 for x in b], dtype=np.uint8)
            out += bytes(b)
        else:
            out += bytes([ws[int(rng.integers(0, 6))] for _ in range(int(rng.integers(1, 4)))])
    return bytes(out[:nbytes])


def score_csv(seed: int = 7, lines: int = 100_000, vocab_size: int = 5_000, split_lines: int = 10_000,
              long_frac: float = 0.01, return_truth: bool = False):
    """``word,score`` lines (a group-by-and-aggregate workload over a CSV
    column): Zipf-distributed words (some longer than 15 bytes), scores with
    three decimals in [-1000, 1000), split into pieces of ``split_lines``
    lines (each ends with a newline).  With ``return_truth`` also
    ``{word: [mean, max, count]}`` of every word that occurs (exact: the
    scores are integers of milli-units)."""
    rng = np.random.default_rng(seed)
    vocab = make_vocab(vocab_size, rng, long_frac=long_frac)
    vocab = [w.replace(b",", b";") for w in vocab]
    cdf = np.cumsum(zipf_probs(vocab_size))
    cdf[-1] = 1.0
    tok = np.minimum(np.searchsorted(cdf, rng.random(lines), side="right"), vocab_size - 1)
    milli = rng.integers(-1_000_000, 1_000_000, lines)
    out = []
    for s0 in range(0, lines, split_lines):
        rows = []
        for t, m in zip(tok[s0:s0 + split_lines], milli[s0:s0 + split_lines]):
            sign = "-" if m < 0 else ""
            a = abs(int(m))
            rows.append(vocab[t] + (",%s%d.%03d\n" % (sign, a // 1000, a % 1000)).encode())
        out.append(b"".join(rows))
    if not return_truth:
        return out
    cnt = np.bincount(tok, minlength=vocab_size)
    tot = np.bincount(tok, weights=milli.astype(np.float64), minlength=vocab_size)
    mx = np.full(vocab_size, np.iinfo(np.int64).min, np.int64)
    np.maximum.at(mx, tok, milli)
    truth = {}
    for i in np.flatnonzero(cnt):
        w = vocab[i].decode("utf-8", "surrogateescape")
        truth[w] = [tot[i] / 1000.0 / cnt[i], mx[i] / 1000.0, int(cnt[i])]
    return out, truth
