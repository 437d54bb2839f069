"""Drop-in for ``bayesian_engine.tiebreak`` (reference src/bayesian_engine/tiebreak.py).

``DeterministicTieBreaker.resolve`` runs the ``bce_tiebreak_csr`` kernel (one wave per
market; CPython ``round(x, precision)`` restated exactly on the GPU, groups in dict
insertion order, input-order sums, lexicographic argmax of (density, max_reliability,
-prediction)).  :meth:`DeterministicTieBreaker.resolve_many` resolves a whole batch of
markets in one launch.  The diagnostics dict is formatted on the host with the same
``round(..., 4)`` / ``round(..., 6)`` calls as the reference (tiebreak.py:136-150).

The empty-list ValueError and the single-agent shortcut (tiebreak.py:86-96) return the
caller's own objects before any compute, as the reference does.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch

from . import _native as N
from . import batch

__all__ = ["TieBreakDiagnostics", "AgentSignal", "DeterministicTieBreaker"]


@dataclass(frozen=True)
class TieBreakDiagnostics:
    """Metadata about tie-break resolution process (tiebreak.py:8-16)."""

    method: str
    groups: Dict[float, Dict]
    selected_group: float
    tie_resolved_by: str
    confidence_variance: float


@dataclass
class AgentSignal:
    """Single agent prediction with metadata (tiebreak.py:19-33)."""

    agent_id: str
    prediction: float
    confidence: float
    weight: float = 1.0
    reliability_score: float = 0.5

    def __post_init__(self):
        if not 0 <= self.confidence <= 1:
            raise ValueError(f"confidence must be in [0,1], got {self.confidence}")
        if not 0 <= self.reliability_score <= 1:
            raise ValueError(f"reliability_score must be in [0,1], got {self.reliability_score}")


class DeterministicTieBreaker:
    """Resolution hierarchy: weight density, then max reliability, then smallest prediction."""

    def __init__(self, precision: int = 6):
        self.precision = precision

    def resolve(self, agents: List[AgentSignal]) -> Tuple[float, TieBreakDiagnostics]:
        if not agents:
            raise ValueError("Cannot resolve tie with empty agent list")
        if len(agents) == 1:
            return agents[0].prediction, TieBreakDiagnostics(
                method="single_agent",
                groups={agents[0].prediction: {"count": 1}},
                selected_group=agents[0].prediction,
                tie_resolved_by="unanimous",
                confidence_variance=0.0,
            )
        return self.resolve_many([agents])[0]

    def _group_keys(self, agents, fkeys, g_of) -> list:
        """The reference's dict keys, round(first member's prediction, precision): the
        kernel's float key, or -- when that first member's prediction is an int -- the
        same value as an int (round(int, n) is an int; tiebreak.py:54)."""
        keys = [float(k) for k in fkeys]
        seen = set()
        for agent, g in zip(agents, g_of):
            g = int(g)
            if g in seen:
                continue
            seen.add(g)
            if isinstance(agent.prediction, int):
                keys[g] = round(agent.prediction, self.precision)
        return keys

    def resolve_many(self, markets: Sequence[Sequence[AgentSignal]]) -> List[Tuple[float, TieBreakDiagnostics]]:
        """resolve() for every market in one kernel launch (empty markets raise)."""
        if any(len(m) == 0 for m in markets):
            raise ValueError("Cannot resolve tie with empty agent list")
        N.require_gpu()
        dev = N.device()
        lens = np.array([len(m) for m in markets], np.int64)
        off = np.zeros(len(markets) + 1, np.int64)
        off[1:] = np.cumsum(lens)
        flat = [a for m in markets for a in m]
        cols = np.array([[float(a.prediction), float(a.confidence), float(a.weight), float(a.reliability_score)]
                         for a in flat], np.float64).reshape(-1, 4)
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        r = batch.tiebreak(T(off), T(cols[:, 0]), T(cols[:, 1]), T(cols[:, 2]), T(cols[:, 3]),
                           precision=int(self.precision), offsets_host=off)
        host = {k: getattr(r, k).cpu().numpy() for k in ("winner", "label", "n_groups", "variance", "g_key",
                                                          "g_count", "g_density", "g_avgconf", "g_maxrel", "g_of")}
        out = []
        for m, agents in enumerate(markets):
            if len(agents) == 1:
                out.append(self.resolve(list(agents)))
                continue
            a = int(off[m])
            ng = int(host["n_groups"][m])
            keys = self._group_keys(agents, host["g_key"][a:a + ng], host["g_of"][a:a + len(agents)])
            groups = {}
            for j, g in enumerate(range(a, a + ng)):
                groups[keys[j]] = {
                    "count": int(host["g_count"][g]),
                    "weight_density": round(float(host["g_density"][g]), 4),
                    "avg_confidence": round(float(host["g_avgconf"][g]), 4),
                    "max_reliability": round(float(host["g_maxrel"][g]), 4),
                }
            wf = float(host["winner"][m])
            winner = next((k for j, k in enumerate(keys) if host["g_key"][a + j] == wf or (wf != wf and k != k)), wf)
            out.append((winner, TieBreakDiagnostics(
                method="prioritized_weight_density",
                groups=groups,
                selected_group=winner,
                tie_resolved_by=N.TB_LABELS[int(host["label"][m])],
                confidence_variance=round(float(host["variance"][m]), 6),
            )))
        return out
