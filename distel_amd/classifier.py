"""ELClassifier / AxiomProcessor mirror over the GPU engine.

The reference runs one JVM per rule type: ``ELClassifier.classify()`` switches on
the ``AxiomDistributionType`` stored in its Redis instance and calls
``TypeXAxiomProcessor.processRules()`` (``kc/ELClassifier.java:65-118``); every
processor implements ``AxiomProcessor.processOneWorkChunk(...) -> boolean``
("some fact was new", ``kc/base/AxiomProcessor.java:14-21``) and all of them
meet at a per-iteration barrier that continues while any processor reported an
update (``kc/controller/CommunicationHandler.java:49-84``).

Here every rule type is a ``GpuAxiomProcessor`` whose
``process_one_work_chunk()`` is one ``el_step(rule)`` on the device (the rule
type's own semi-naive delta, like the reference's per-type score watermarks).
``ELClassifier.classify("rule-types")`` reproduces the reference's schedule
(all eight types per iteration, barrier, repeat while anything changed);
``classify("fused")`` runs ``el_saturate`` — the same fixpoint with all rule
types fused into each Jacobi superstep, which is the fast path.
Errors surface as ``ElError`` (the reference's ``throws Exception``).
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional

from .engine import AxiomDistributionType, Engine, ElError, Stats
from .ir import Axioms


class AxiomProcessor:
    """``kc/base/AxiomProcessor.java:14-21``."""

    def process_one_work_chunk(self) -> bool:  # pragma: no cover - interface
        raise NotImplementedError

    def send_progress_message(self, progress: float, iteration_count: int) -> None:
        """Progress gossip over PUB/SUB in the reference (work stealing); nothing to do on one device."""

    def clean_up(self) -> None:
        pass


class GpuAxiomProcessor(AxiomProcessor):
    """One rule type's entry point on the device (``el_step``)."""

    def __init__(self, engine: Engine, axiom_type: AxiomDistributionType):
        self.engine = engine
        self.axiom_type = AxiomDistributionType(axiom_type)

    def process_one_work_chunk(self) -> bool:
        return self.engine.step(self.axiom_type)


class ELClassifier:
    """Loads the normalized axioms once (AxiomLoader), then classifies (ELClassifier)."""

    def __init__(self, axioms: Axioms, device: int = 0, profile: bool = False, compat_chain: bool = False):
        self.axioms = axioms
        self.engine = Engine(device=device, profile=profile, compat_chain=compat_chain)
        t0 = time.perf_counter()
        self.engine.load(axioms)
        self.engine.init()
        self.load_ms = 1e3 * (time.perf_counter() - t0)
        self.processors: Dict[AxiomDistributionType, GpuAxiomProcessor] = {
            t: GpuAxiomProcessor(self.engine, t) for t in AxiomDistributionType}
        self.iterations: List[Dict[str, bool]] = []

    def classify(self, mode: str = "fused") -> Stats:
        if mode == "fused":
            return self.engine.saturate()
        if mode != "rule-types":
            raise ValueError("mode must be 'fused' or 'rule-types'")
        t0 = time.perf_counter()
        next_iteration = True
        while next_iteration:
            status = {t.name: p.process_one_work_chunk() for t, p in self.processors.items()}
            self.iterations.append(status)
            next_iteration = any(status.values())  # CommunicationHandler: continue if any update
        st = self.engine.stats()
        st["ms"] = 1e3 * (time.perf_counter() - t0)
        st["supersteps"] = len(self.iterations)
        return st

    def close(self) -> None:
        for p in self.processors.values():
            p.clean_up()
        self.engine.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
