"""Token sampling for the HTTP front end: llama-server's default sampler chain.

The reference's backend is llama-server (scripts/start.sh:235); its request fields
temperature / top_p / frequency_penalty / presence_penalty / stop are documented in
docs/API_REFERENCE.md:363-379 and forwarded verbatim by scripts/gateway.py:699-804.
Upstream llama-server (not vendored) samples each token with the chain

    penalties -> top_k -> top_p -> min_p -> temperature -> dist

restated here on the host over the logits of llama_get_logits_ith:

  penalties  for every token t among the last `repeat_last_n` generated/prompt tokens,
             with c = its count there: logit <= 0 ? logit * repeat_penalty
             : logit / repeat_penalty, then logit -= c * frequency_penalty +
             presence_penalty
  top_k      keep the k largest logits (k <= 0: all)
  top_p      softmax over the kept ones, keep the smallest prefix (by logit, descending)
             whose probability mass reaches p (at least one)
  min_p      keep the tokens with p >= min_p * p_max
  temp       logits / temperature; temperature <= 0 keeps only the largest (greedy,
             first max wins as llama_sampler_greedy)
  dist       softmax, one draw from a seeded generator (per request; seed < 0 or
             absent: a fresh random seed)

Defaults are llama-server's (temperature 0.8, top_k 40, top_p 0.95, min_p 0.05,
repeat_penalty 1.0 over the last 64 tokens, no frequency/presence penalty); the server's
--temp/--top-k/... flags change them as llama-server's do.  Requests whose chain reduces
to an argmax of the raw logits (temperature <= 0 or top_k == 1, no penalties) decode on
the device (llmi_generate_greedy_batch) with no logits copy.  The random stream is
numpy's PCG64, not llama.cpp's mt19937: sampled text with a given seed is reproducible
here but not token-identical to llama-server's (parity of sampled output is unpinned;
greedy output is the parity bar, tests/test_gpu_*.py).
"""
from __future__ import annotations

from dataclasses import dataclass, replace
from typing import Optional, Sequence

import numpy as np


@dataclass(frozen=True)
class SamplingParams:
    temperature: float = 0.8
    top_k: int = 40
    top_p: float = 0.95
    min_p: float = 0.05
    repeat_penalty: float = 1.0
    repeat_last_n: int = 64
    presence_penalty: float = 0.0
    frequency_penalty: float = 0.0
    seed: int = -1

    @property
    def penalized(self) -> bool:
        return self.repeat_penalty != 1.0 or self.presence_penalty != 0.0 or self.frequency_penalty != 0.0

    @property
    def greedy(self) -> bool:
        """The whole chain is an argmax of the raw logits (the device fast path)."""
        return (self.temperature <= 0.0 or self.top_k == 1) and not self.penalized

    def with_request(self, req: dict) -> "SamplingParams":
        """These defaults overridden by a request's fields (llama-server / OpenAI names);
        ValueError for a value llama-server would reject."""
        kw = {}

        def num(name, cast, lo=None, hi=None, alias=None):
            v = req.get(name, req.get(alias) if alias else None)
            if v is None:
                return
            if isinstance(v, bool) or not isinstance(v, (int, float)):
                raise ValueError(f"'{name}' must be a number")
            v = cast(v)
            if (lo is not None and v < lo) or (hi is not None and v > hi):
                raise ValueError(f"'{name}' out of range [{lo}, {hi}]")
            kw[name] = v

        num("temperature", float, 0.0, 100.0)
        num("top_k", int, None, None)
        num("top_p", float, 0.0, 1.0)
        num("min_p", float, 0.0, 1.0)
        num("repeat_penalty", float, 0.0, None)
        num("repeat_last_n", int, -1, None)
        num("presence_penalty", float, -2.0, 2.0)
        num("frequency_penalty", float, -2.0, 2.0)
        num("seed", int, None, None)
        return replace(self, **kw)


def _softmax(x: np.ndarray) -> np.ndarray:
    e = np.exp(x - x.max())
    return e / e.sum()


class Sampler:
    """One request's sampler (its own generator)."""

    def __init__(self, params: SamplingParams):
        self.p = params
        self.rng = np.random.default_rng(params.seed if params.seed >= 0 else None)

    def sample(self, logits: np.ndarray, history: Sequence[int]) -> int:
        p = self.p
        lg = np.array(logits, dtype=np.float32, copy=True)
        if p.penalized:
            n = len(history) if p.repeat_last_n < 0 else min(p.repeat_last_n, len(history))
            if n > 0:
                toks, counts = np.unique(np.asarray(history[len(history) - n:], dtype=np.int64), return_counts=True)
                toks, counts = toks[(toks >= 0) & (toks < lg.size)], counts[(toks >= 0) & (toks < lg.size)]
                v = lg[toks]
                v = np.where(v <= 0, v * p.repeat_penalty, v / p.repeat_penalty)
                v = v - counts * p.frequency_penalty - (counts > 0) * p.presence_penalty
                lg[toks] = v.astype(np.float32)
        if p.temperature <= 0.0:
            return int(np.argmax(lg))
        # candidates sorted by logit, descending (stable: lower ids first on ties)
        k = lg.size if p.top_k <= 0 else min(p.top_k, lg.size)
        if k < lg.size:
            idx = np.argpartition(-lg, k - 1)[:k]
        else:
            idx = np.arange(lg.size)
        idx = idx[np.lexsort((idx, -lg[idx]))]
        cand = lg[idx].astype(np.float64)
        if p.top_p < 1.0:
            pr = _softmax(cand)
            keep = int(np.searchsorted(np.cumsum(pr), p.top_p) + 1)
            idx, cand = idx[:max(1, keep)], cand[:max(1, keep)]
        if p.min_p > 0.0 and cand.size > 1:
            pr = _softmax(cand)
            m = pr >= p.min_p * pr[0]
            m[0] = True
            idx, cand = idx[m], cand[m]
        pr = _softmax(cand / p.temperature)
        return int(idx[self.rng.choice(pr.size, p=pr)])


def find_stop(text: str, stops: Sequence[str]) -> Optional[int]:
    """Index of the earliest occurrence of any stop string in text, or None."""
    best = None
    for s in stops:
        if s:
            i = text.find(s)
            if i >= 0 and (best is None or i < best):
                best = i
    return best


class StopFilter:
    """Streams text while holding back any tail that could still begin a stop string;
    `done` truncates at the stop string (llama-server's partial-stop handling)."""

    def __init__(self, stops: Sequence[str]):
        self.stops = [s for s in stops if s]
        self.hold = max((len(s) for s in self.stops), default=1) - 1
        self.text = ""
        self.sent = 0
        self.stopped = False

    def push(self, piece: str) -> str:
        if self.stopped:
            return ""
        self.text += piece
        i = find_stop(self.text, self.stops)
        if i is not None:
            self.stopped = True
            out = self.text[self.sent:i]
            self.sent = i
            return out
        safe = max(self.sent, len(self.text) - self.hold)
        out = self.text[self.sent:safe]
        self.sent = safe
        return out

    def flush(self) -> str:
        if self.stopped:
            return ""
        out = self.text[self.sent:]
        self.sent = len(self.text)
        return out


def parse_stop(v) -> list[str]:
    if v is None:
        return []
    if isinstance(v, str):
        return [v]
    if isinstance(v, list) and all(isinstance(s, str) for s in v):
        return list(v)
    raise ValueError("'stop' must be a string or a list of strings")
