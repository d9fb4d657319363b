"""Command line: the reference's load / classify / diff scripts over the GPU engine.

  python -m distel_amd.cli classify ONTOLOGY.ofn [--normalized] [--out FILE] [--names]
                                    [--parts N] [--device D] [--layout x2b|b2x]
      = AxiomLoader <ontology> <isNormalized> (kc/init/AxiomLoader.java:1380-1392)
        + classify-all.sh (ELClassifier per rule type) + ResultRearranger +
        ELClassifierTest.writeResultsToFile (``X|B`` lines, kc/test/ELClassifierTest.java:448-469)
  python -m distel_amd.cli normalize IN.ofn OUT.ofn
      = Normalizer.main (kc/init/Normalizer.java:920-959), functional syntax out
  python -m distel_amd.cli diff EXPECTED.txt RESULT.txt
      = ResultDiffWriter / the comparison of test-classify.sh: both files hold ``X|B`` lines
        (e.g. an ELK taxonomy dumped the same way on a machine with a JVM)
Times: load (parse + normalize + index upload) and classification are reported apart,
as run-all.sh does (scripts/run-all.sh:24-27).
"""
from __future__ import annotations

import argparse
import json
import sys
import time


def _classify(args) -> int:
    from . import engine, owl
    from .result import ResultNode
    t0 = time.perf_counter()
    ax = owl.load_functional(args.ontology, normalized=args.normalized)
    parse_s = time.perf_counter() - t0
    if args.parts > 1:
        if args.compat_chain:
            raise SystemExit("--compat-chain runs on one context (--parts 1)")
        t1 = time.perf_counter()
        engs, sts = engine.classify_partitioned(ax, args.parts, devices=list(range(args.devices)))
        cls_s = time.perf_counter() - t1
        fx, fa = engine.merge_facts(engs)
        derived = sum(s["derived"] for s in sts)
        steps = sts[0]["supersteps"]
        for e in engs:
            e.close()
    else:
        eng = engine.Engine(device=args.device, compat_chain=args.compat_chain)
        t1 = time.perf_counter()
        eng.load(ax)
        load_s = time.perf_counter() - t1
        t1 = time.perf_counter()
        eng.init()
        st = eng.saturate()
        cls_s = time.perf_counter() - t1
        fx, fa = eng.facts()
        derived, steps = st["derived"], st["supersteps"]
        eng.close()
    rn = ResultNode(ax, fx, fa, distel_compat=args.distel_compat)
    n = rn.write_saxioms(args.out, use_names=args.names) if args.out else 0
    print(json.dumps({"concepts": ax.n_concepts, "roles": ax.n_roles, "axioms": ax.counts(),
                      "parse_normalize_s": round(parse_s, 3), "classification_s": round(cls_s, 6),
                      "supersteps": steps, "derived": derived, "saxioms_written": n}))
    return 0


def _normalize(args) -> int:
    from . import owl
    with open(args.input, encoding="utf-8") as f:
        onto = owl.parse_functional(f.read())
    n = owl.write_functional(owl.normalize(onto), args.output)
    print(f"No of axioms after normalization: {n}")
    return 0


def _diff(args) -> int:
    from .result import diff_results, read_saxioms
    misses, report = diff_results(read_saxioms(args.expected), read_saxioms(args.result), bottom=args.bottom)
    print("\n".join(report))
    return 1 if misses else 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="distel_amd.cli")
    sub = ap.add_subparsers(dest="cmd", required=True)
    c = sub.add_parser("classify")
    c.add_argument("ontology")
    c.add_argument("--normalized", action="store_true", help="input is already normalized (isNormalized=true)")
    c.add_argument("--out", help="write X|B lines here")
    c.add_argument("--names", action="store_true", help="IRIs instead of DistEL packed ids")
    c.add_argument("--distel-compat", action="store_true", help="add individuals' ⊥ ⊑ a entries (H7)")
    c.add_argument("--compat-chain", action="store_true",
                   help="DistEL's CR6 join that ignores s (hazard H2, EL_FLAG_COMPAT_DISTEL_CHAIN)")
    c.add_argument("--device", type=int, default=0)
    c.add_argument("--parts", type=int, default=1, help="row partitions (in-process delta exchange)")
    c.add_argument("--devices", type=int, default=1, help="GPUs the partitions are spread over")
    c.set_defaults(fn=_classify)
    n = sub.add_parser("normalize")
    n.add_argument("input")
    n.add_argument("output")
    n.set_defaults(fn=_normalize)
    d = sub.add_parser("diff")
    d.add_argument("expected")
    d.add_argument("result")
    d.add_argument("--bottom", default=None, help="name of ⊥ in both files (default: owl:Nothing / its IRI)")
    d.set_defaults(fn=_diff)
    args = ap.parse_args(argv)
    return args.fn(args)


if __name__ == "__main__":
    sys.exit(main())
