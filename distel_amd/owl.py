"""OWL 2 functional-syntax loader and EL+ normalizer.

DistEL's ``AxiomLoader`` (``kc/init/AxiomLoader.java:126-207``) reads an ontology with
OWLAPI, optionally normalizes it (``Normalizer.Normalize``, ``kc/init/Normalizer.java:
117-208``), types every normalized axiom into one rule family
(``categorizeAxiomsIntoTypes`` :495-577) and numbers the entities
(``mapConceptToID`` :1155-1341).  This module does the same for OWL 2 functional
syntax — the format DistEL's Normalizer and OntologyMultiplier save
(``Normalizer.java:954-959``, ``OntologyMultiplier.java:84-85``) — and yields the typed
``ir.Axioms`` the engine's ``el_load`` takes, with the IRI of every concept and role.

Class expressions (the reference's accepted EL+ fragment, ``Normalizer.isAcceptableType``
:347-365 and ``AxiomLoader.isClass / isExistential`` :579-595):

* named classes, ``owl:Thing``, ``owl:Nothing``;
* ``ObjectOneOf(a)`` with one individual (more than one: skipped, H6 — ``AxiomLoader.java:
  1003-1012``);
* ``ObjectIntersectionOf``, ``ObjectSomeValuesFrom``, ``ObjectHasValue(r a)`` = ∃r.{a};
* ``DataSomeValuesFrom(p DT)`` and ``DataHasValue(p "v"^^DT)``: the datatype becomes a
  concept of kind DATATYPE (``conceptToIDForDataType``, ``AxiomLoader.java:783-800``).

Axioms: SubClassOf, EquivalentClasses, DisjointClasses (pairwise A ⊓ B ⊑ ⊥), ClassAssertion,
ObjectPropertyAssertion, DataPropertyAssertion, SubObjectPropertyOf (incl.
ObjectPropertyChain), SubDataPropertyOf, EquivalentObjectProperties, TransitiveObjectProperty
(r ∘ r ⊑ r, ``Normalizer.java:294-308``), Object/DataPropertyDomain, ObjectPropertyRange.
Everything else (annotations, declarations, functional/inverse/... property axioms) carries
no EL+ consequence and is counted in ``Ontology.skipped``.

Normalization (``normalize``) applies NF1-NF7 (``Normalizer.java:500-784``) exhaustively,
with range elimination ("Pushing the EL Envelope Further", ``Normalizer.java:119-137,
455-497``): the result has only the four normal forms A ⊑ B, A1 ⊓ A2 ⊑ B, A ⊑ ∃r.B,
∃r.A ⊑ B plus role axioms.  Fresh classes/properties are named deterministically
(``urn:distel-amd:gensym#C<n>`` / ``#R<n>``) in first-use order, and one complex expression
always gets the same fresh class (``checkAndCreateConcept`` :892-918, whose Redis cache this
replaces) — the reference uses random UUIDs, so its fresh names are not reproducible.
"""
from __future__ import annotations

import re
import warnings
from collections import Counter
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Tuple, Union

from . import ir

OWL = "http://www.w3.org/2002/07/owl#"
THING = OWL + "Thing"
NOTHING = OWL + "Nothing"
XSD_STRING = "http://www.w3.org/2001/XMLSchema#string"
RDF_PLAIN = "http://www.w3.org/1999/02/22-rdf-syntax-ns#PlainLiteral"
GENSYM = "urn:distel-amd:gensym#"
DEFAULT_PREFIXES = {
    "owl": OWL,
    "rdf": "http://www.w3.org/1999/02/22-rdf-syntax-ns#",
    "rdfs": "http://www.w3.org/2000/01/rdf-schema#",
    "xsd": "http://www.w3.org/2001/XMLSchema#",
    "xml": "http://www.w3.org/XML/1998/namespace",
}

# ------------------------------------------------------------------ expressions
# Class expressions are hashable tuples:
#   ("C", iri)                named class (owl:Thing / owl:Nothing included)
#   ("I", iri)                ObjectOneOf with one individual: {a}
#   ("D", iri)                a datatype, as the filler of a data existential
#   ("AND", frozenset(...))   ObjectIntersectionOf
#   ("SOME", role_iri, expr)  Object/DataSomeValuesFrom, ObjectHasValue, DataHasValue
#   ("ONEOF", frozenset(iris))  ObjectOneOf with several individuals (unsupported, H6)
Expr = tuple
TOP_E: Expr = ("C", THING)
BOT_E: Expr = ("C", NOTHING)


def is_basic(e: Expr) -> bool:
    """``Normalizer.isBasic`` (:870-878): classes, ⊤, ⊥, individuals (and datatypes)."""
    return e[0] in ("C", "I", "D")


@dataclass
class Ontology:
    """Parsed axioms in the shape DistEL's loader works on."""
    sub: List[Tuple[Expr, Expr]] = field(default_factory=list)          # C ⊑ D
    subrole: List[Tuple[str, str]] = field(default_factory=list)        # r ⊑ s
    chain: List[Tuple[Tuple[str, ...], str]] = field(default_factory=list)  # r1 ∘ … ∘ rn ⊑ s
    domain: List[Tuple[str, Expr]] = field(default_factory=list)
    range: List[Tuple[str, Expr]] = field(default_factory=list)
    classes: set = field(default_factory=set)
    individuals: set = field(default_factory=set)
    object_props: set = field(default_factory=set)
    data_props: set = field(default_factory=set)
    datatypes: set = field(default_factory=set)
    skipped: Counter = field(default_factory=Counter)
    iri: Optional[str] = None


# ------------------------------------------------------------------ tokenizer / parser
_TOKEN = re.compile(r"""
    (?P<ws>\s+|\#[^\n]*)
  | (?P<iri><[^>]*>)
  | (?P<str>"(?:[^"\\]|\\.)*")
  | (?P<lp>\()
  | (?P<rp>\))
  | (?P<eq>=)
  | (?P<tt>\^\^)
  | (?P<lang>@[A-Za-z][A-Za-z0-9-]*)
  | (?P<name>[^\s()"<>=^@][^\s()"<>=^]*)
""", re.X)


class ParseError(ValueError):
    pass


def _tokens(text: str):
    pos, n = 0, len(text)
    while pos < n:
        m = _TOKEN.match(text, pos)
        if not m:
            raise ParseError(f"unexpected character at offset {pos}: {text[pos:pos + 20]!r}")
        pos = m.end()
        kind = m.lastgroup
        if kind == "ws":
            continue
        yield kind, m.group(kind)


class _Lit:
    __slots__ = ("value", "datatype")

    def __init__(self, value: str, datatype: str):
        self.value, self.datatype = value, datatype


def _sexpr(text: str) -> List:
    """Functional syntax → nested lists: [head, arg, ...]; IRIs/names stay str, literals _Lit."""
    root: List = []
    stack: List[List] = [root]
    prev = None
    toks = list(_tokens(text))
    i = 0
    while i < len(toks):
        kind, v = toks[i]
        if kind == "lp":
            if not stack[-1] or not isinstance(stack[-1][-1], str):
                raise ParseError("'(' must follow a keyword")
            head = stack[-1].pop()
            node = [head]
            stack[-1].append(node)
            stack.append(node)
        elif kind == "rp":
            if len(stack) == 1:
                raise ParseError("unbalanced ')'")
            stack.pop()
        elif kind == "str":
            val = bytes(v[1:-1], "utf-8").decode("unicode_escape") if "\\" in v else v[1:-1]
            dt = RDF_PLAIN
            if i + 1 < len(toks) and toks[i + 1][0] == "tt":
                dt = toks[i + 2][1]
                i += 2
            elif i + 1 < len(toks) and toks[i + 1][0] == "lang":
                i += 1
            stack[-1].append(_Lit(val, dt))
        elif kind == "eq":
            stack[-1].append("=")
        elif kind in ("iri", "name"):
            stack[-1].append(v)
        else:
            raise ParseError(f"unexpected token {v!r}")
        i += 1
    if len(stack) != 1:
        raise ParseError("unbalanced '('")
    return root


class _Reader:
    def __init__(self):
        self.prefixes = dict(DEFAULT_PREFIXES)
        self.o = Ontology()

    def iri(self, t) -> str:
        if isinstance(t, _Lit):
            raise ParseError(f"expected an IRI, got literal {t.value!r}")
        if t.startswith("<"):
            return t[1:-1]
        if ":" in t:
            p, local = t.split(":", 1)
            if p in self.prefixes:
                return self.prefixes[p] + local
            raise ParseError(f"unknown prefix {p!r} in {t!r}")
        raise ParseError(f"not an IRI: {t!r}")

    def lit_iri(self, t) -> str:
        if isinstance(t, _Lit):
            return self.iri(t.datatype) if not t.datatype.startswith("http") else t.datatype
        return self.iri(t)

    # -- class expressions
    def ce(self, t) -> Expr:
        if isinstance(t, str):
            c = self.iri(t)
            if c not in (THING, NOTHING):
                self.o.classes.add(c)
            return ("C", c)
        head, args = t[0], t[1:]
        if head == "ObjectIntersectionOf":
            ops = frozenset(self.ce(a) for a in args)
            if not ops:
                return TOP_E
            return next(iter(ops)) if len(ops) == 1 else ("AND", ops)
        if head == "ObjectSomeValuesFrom":
            r = self.oprop(args[0])
            return ("SOME", r, self.ce(args[1]))
        if head == "ObjectHasValue":
            r = self.oprop(args[0])
            return ("SOME", r, ("I", self.ind(args[1])))
        if head == "ObjectOneOf":
            inds = frozenset(self.ind(a) for a in args)
            return ("I", next(iter(inds))) if len(inds) == 1 else ("ONEOF", inds)
        if head == "DataSomeValuesFrom":
            if len(args) != 2:
                raise _Unsupported("DataSomeValuesFrom/n-ary")
            p = self.dprop(args[0])
            dr = args[1]
            if not isinstance(dr, str):
                raise _Unsupported(f"DataSomeValuesFrom/{dr[0]}")
            return ("SOME", p, self.dt(self.iri(dr)))
        if head == "DataHasValue":
            p = self.dprop(args[0])
            return ("SOME", p, self.dt(self.lit_iri(args[1])))
        raise _Unsupported(head)

    def dt(self, iri: str) -> Expr:
        self.o.datatypes.add(iri)
        return ("D", iri)

    def ind(self, t) -> str:
        a = self.iri(t)
        self.o.individuals.add(a)
        return a

    def oprop(self, t) -> str:
        if not isinstance(t, str):
            raise _Unsupported(f"property expression {t[0]}")  # ObjectInverseOf is outside EL+
        r = self.iri(t)
        self.o.object_props.add(r)
        return r

    def dprop(self, t) -> str:
        p = self.iri(t)
        self.o.data_props.add(p)
        return p

    # -- axioms
    def axiom(self, t) -> None:
        head, args = t[0], t[1:]
        args = [a for a in args if not (isinstance(a, list) and a[0] == "Annotation")]
        o = self.o
        if head == "Declaration":
            kind, name = args[0][0], self.iri(args[0][1])
            if kind == "Class" and name in (THING, NOTHING):
                return
            {"Class": o.classes, "NamedIndividual": o.individuals, "ObjectProperty": o.object_props,
             "DataProperty": o.data_props, "Datatype": o.datatypes}.get(kind, set()).add(name)
        elif head == "SubClassOf":
            o.sub.append((self.ce(args[0]), self.ce(args[1])))
        elif head == "EquivalentClasses":
            es = [self.ce(a) for a in args]
            for i, a in enumerate(es):  # OWLAPI asOWLSubClassOfAxioms: every ordered pair
                for b in es[i + 1:]:
                    o.sub.append((a, b))
                    o.sub.append((b, a))
        elif head == "DisjointClasses":
            es = [self.ce(a) for a in args]
            for i, a in enumerate(es):
                for b in es[i + 1:]:
                    o.sub.append((("AND", frozenset((a, b))), BOT_E))
        elif head == "ClassAssertion":
            o.sub.append((("I", self.ind(args[1])), self.ce(args[0])))
        elif head == "ObjectPropertyAssertion":
            r = self.oprop(args[0])
            o.sub.append((("I", self.ind(args[1])), ("SOME", r, ("I", self.ind(args[2])))))
        elif head == "DataPropertyAssertion":
            p = self.dprop(args[0])
            o.sub.append((("I", self.ind(args[1])), ("SOME", p, self.dt(self.lit_iri(args[2])))))
        elif head == "SubObjectPropertyOf":
            sup = self.oprop(args[1])
            if isinstance(args[0], list) and args[0][0] == "ObjectPropertyChain":
                o.chain.append((tuple(self.oprop(a) for a in args[0][1:]), sup))
            else:
                o.subrole.append((self.oprop(args[0]), sup))
        elif head == "SubDataPropertyOf":
            o.subrole.append((self.dprop(args[0]), self.dprop(args[1])))
        elif head == "EquivalentObjectProperties":
            rs = [self.oprop(a) for a in args]
            for a in rs:
                for b in rs:
                    if a != b:
                        o.subrole.append((a, b))
        elif head == "TransitiveObjectProperty":
            r = self.oprop(args[0])
            o.chain.append(((r, r), r))
        elif head in ("ObjectPropertyDomain", "DataPropertyDomain"):
            r = self.oprop(args[0]) if head[0] == "O" else self.dprop(args[0])
            o.domain.append((r, self.ce(args[1])))
        elif head == "ObjectPropertyRange":
            r = self.oprop(args[0])
            rng = args[1]
            if isinstance(rng, list) and rng[0] == "ObjectUnionOf":  # AxiomLoader.java:860-861
                o.skipped["ObjectPropertyRange/ObjectUnionOf"] += 1
                return
            o.range.append((r, self.ce(rng)))
        else:
            o.skipped[head] += 1

    def document(self, root: List) -> Ontology:
        for node in root:
            if not isinstance(node, list):
                if node == "=":
                    continue
                raise ParseError(f"unexpected top-level token {node!r}")
            if node[0] == "Prefix":
                body = [x for x in node[1:] if x != "="]
                name = body[0]
                if not name.endswith(":"):
                    raise ParseError(f"bad prefix declaration {body}")
                self.prefixes[name[:-1]] = body[1][1:-1]
            elif node[0] == "Ontology":
                for ax in node[1:]:
                    if isinstance(ax, str):  # ontology / version IRI
                        if self.o.iri is None:
                            self.o.iri = self.iri(ax)
                        continue
                    if ax[0] in ("Import", "Annotation"):
                        self.o.skipped[ax[0]] += 1
                        continue
                    try:
                        self.axiom(ax)
                    except _Unsupported as u:
                        self.o.skipped[f"{ax[0]}/{u}"] += 1
            else:
                raise ParseError(f"unexpected top-level element {node[0]!r}")
        return self.o


class _Unsupported(Exception):
    pass


def parse_functional(text: str) -> Ontology:
    """Parse an OWL 2 functional-syntax document (``Prefix(...) Ontology(...)``)."""
    return _Reader().document(_sexpr(text))


# ------------------------------------------------------------------ normalizer
class Normalizer:
    """NF1-NF7 + range elimination (``kc/init/Normalizer.java``), deterministic gensyms."""

    def __init__(self, onto: Ontology):
        self.o = onto
        self.names: Dict[Expr, Expr] = {}   # checkAndCreateConcept: expression -> fresh class
        self.nc = 0
        self.nr = 0
        self.out = Ontology(classes=set(onto.classes), individuals=set(onto.individuals),
                            object_props=set(onto.object_props), data_props=set(onto.data_props),
                            datatypes=set(onto.datatypes), skipped=Counter(onto.skipped), iri=onto.iri)
        # object property ranges, eliminated (Normalizer.java:119-137)
        self.ranges: Dict[str, List[Expr]] = {}
        for r, c in onto.range:
            if c[0] != "C":
                self.out.skipped["ObjectPropertyRange/complex"] += 1
                continue
            self.ranges.setdefault(r, []).append(c)
        self.range_repl: Dict[Tuple[str, Expr], Expr] = {}
        self.hits = 0

    def fresh_class(self) -> Expr:
        self.nc += 1
        c = f"{GENSYM}C{self.nc}"
        self.out.classes.add(c)
        return ("C", c)

    def fresh_role(self) -> str:
        self.nr += 1
        r = f"{GENSYM}R{self.nr}"
        self.out.object_props.add(r)
        return r

    def name(self, e: Expr) -> Expr:
        """``checkAndCreateConcept`` (Normalizer.java:892-918)."""
        n = self.names.get(e)
        if n is None:
            n = self.names[e] = self.fresh_class()
        else:
            self.hits += 1
        return n

    @staticmethod
    def acceptable(e: Expr) -> bool:
        """``isAcceptableType`` (Normalizer.java:347-365), plus data existentials."""
        if e[0] == "ONEOF":
            return False
        if e[0] == "AND":
            return all(Normalizer.acceptable(x) for x in e[1])
        if e[0] == "SOME":
            return Normalizer.acceptable(e[2])
        return True

    def run(self) -> Ontology:
        for sub, sup in self.o.sub:
            if not (self.acceptable(sub) and self.acceptable(sup)):
                self.out.skipped["SubClassOf/ObjectOneOf(n>1)"] += 1  # H6
                continue
            self.sub(sub, sup)
        for r, s in self.o.subrole:
            self.out.subrole.append((r, s))
        for chain, s in self.o.chain:
            self.chain(list(chain), s)
        for r, d in self.o.domain:
            if is_basic(d):
                self.out.domain.append((r, d))
            else:  # complex domain: ∃r.⊤ ⊑ D
                self.sub(("SOME", r, TOP_E), d)
        return self.out

    def chain(self, props: List[str], s: str) -> None:
        """NF1 (Normalizer.java:619-638): r1 ∘ … ∘ rn ⊑ s into binary chains."""
        if len(props) == 1:
            self.out.subrole.append((props[0], s))
            return
        if len(props) == 2:
            self.out.chain.append((tuple(props), s))
            return
        u = self.fresh_role()
        self.chain(props[:-1], u)
        self.out.chain.append(((u, props[-1]), s))

    def some_rhs(self, b: Expr, r: str, f: Expr) -> None:
        """B ⊑ ∃r.F (F basic), with range elimination (eliminateObjPropertyRange :455-497)."""
        rngs = self.ranges.get(r)
        if not rngs or f[0] == "D":
            self.out.sub.append((b, ("SOME", r, f)))
            return
        key = (r, f)
        x = self.range_repl.get(key)
        if x is None:
            x = self.range_repl[key] = self.fresh_class()
            self.out.sub.append((x, f))
            for c in rngs:
                self.out.sub.append((x, c))
        self.out.sub.append((b, ("SOME", r, x)))

    def sub(self, c: Expr, d: Expr) -> None:
        if c == BOT_E:                                   # NF4: ⊥ ⊑ D is trivial
            return
        if d == TOP_E:                                   # C ⊑ ⊤ is trivial
            return
        if is_basic(c):
            if is_basic(d):
                self.out.sub.append((c, d))
            elif d[0] == "AND":                          # NF7
                for x in sorted(d[1], key=repr):
                    self.sub(c, x)
            elif d[0] == "SOME":
                f = d[2]
                if is_basic(f):
                    self.some_rhs(c, d[1], f)
                else:                                    # NF6
                    a = self.name(f)
                    self.some_rhs(c, d[1], a)
                    self.sub(a, f)
            return
        if not is_basic(d):                              # NF5
            a = self.name(c)
            self.sub(c, a)
            self.sub(a, d)
            return
        if c[0] == "AND":                                # NF2 (+ NF8 binarisation)
            ops = sorted(c[1], key=repr)
            basic = []
            for op in ops:
                if is_basic(op):
                    basic.append(op)
                else:
                    a = self.name(op)
                    self.sub(op, a)
                    basic.append(a)
            basic = sorted(set(basic), key=repr)
            if TOP_E in basic and len(basic) > 1:
                basic.remove(TOP_E)
            if len(basic) == 1:
                self.sub(basic[0], d)
            elif len(basic) == 2:
                self.out.sub.append((("AND", frozenset(basic)), d))
            else:
                rest = ("AND", frozenset(basic[1:]))
                x = self.name(rest)
                self.sub(rest, x)
                self.out.sub.append((("AND", frozenset((basic[0], x))), d))
            return
        if c[0] == "SOME":                               # NF3
            f = c[2]
            if is_basic(f):
                self.out.sub.append((c, d))
            else:
                a = self.name(f)
                self.sub(f, a)
                self.out.sub.append((("SOME", c[1], a), d))
            return
        raise ValueError(f"cannot normalize {c!r} ⊑ {d!r}")


def normalize(onto: Ontology) -> Ontology:
    return Normalizer(onto).run()


# ------------------------------------------------------------------ typing → IR
def to_axioms(onto: Ontology) -> ir.Axioms:
    """Type a normalized ontology into the rule families (``categorizeAxiomsIntoTypes``,
    AxiomLoader.java:495-577) over dense ids: ⊥ = 0, ⊤ = 1, then classes, individuals and
    datatypes in IRI order; roles = object then data properties in IRI order."""
    b = ir._Builder()
    b.cnames[ir.BOTTOM], b.cnames[ir.TOP] = NOTHING, THING
    b.concepts = {NOTHING: ir.BOTTOM, THING: ir.TOP}
    for c in sorted(onto.classes - {THING, NOTHING}):
        b.c(c, ir.KIND_CLASS, True)
    for a in sorted(onto.individuals):
        b.c(a, ir.KIND_INDIVIDUAL, True)
    for d in sorted(onto.datatypes):
        b.c(d, ir.KIND_DATATYPE, True)
    for r in sorted(onto.object_props) + sorted(onto.data_props - onto.object_props):
        b.r(r)

    def cid(e: Expr) -> int:
        if e[0] == "C":
            return b.c(e[1], ir.KIND_CLASS)
        if e[0] == "I":
            return b.c(e[1], ir.KIND_INDIVIDUAL)
        if e[0] == "D":
            return b.c(e[1], ir.KIND_DATATYPE)
        raise ValueError(f"not a basic concept: {e!r}")

    for c, d in onto.sub:
        if d == TOP_E or c == BOT_E:
            continue
        if is_basic(c):
            if is_basic(d):
                b.sub.append((cid(c), cid(d)))                       # CR_TYPE1_1
            elif d[0] == "SOME" and is_basic(d[2]):
                b.ex_rhs.append((cid(c), b.r(d[1]), cid(d[2])))      # CR_TYPE2
            else:
                raise ValueError(f"axiom not in normal form: {c!r} ⊑ {d!r} (normalize first)")
        elif c[0] == "AND" and all(is_basic(x) for x in c[1]) and is_basic(d):
            b.conj.append((sorted(cid(x) for x in c[1]), cid(d)))    # CR_TYPE1_2
        elif c[0] == "SOME" and is_basic(c[2]) and is_basic(d):
            b.ex_lhs.append((b.r(c[1]), cid(c[2]), cid(d)))          # CR_TYPE3_1
        else:
            raise ValueError(f"axiom not in normal form: {c!r} ⊑ {d!r} (normalize first)")
    for r, s in onto.subrole:
        b.subrole.append((b.r(r), b.r(s)))                           # CR_TYPE4
    for chain, s in onto.chain:
        if len(chain) != 2:  # AxiomLoader.java:1108-1110 throws on longer chains
            raise ValueError(f"role chain of length {len(chain)} (normalize first)")
        b.chain.append((b.r(chain[0]), b.r(chain[1]), b.r(s)))       # CR_TYPE5
    for r, d in onto.domain:
        if not is_basic(d):
            raise ValueError("complex property domain (normalize first)")
        b.domain.append((b.r(r), cid(d)))
    for r, c in onto.range:
        if c[0] != "C":
            continue
        b.range.append((b.r(r), cid(c)))
    return b.axioms()


def load_functional(path: str, normalized: bool = False) -> ir.Axioms:
    """``AxiomLoader(<ontology>, isNormalized)``: parse, normalize unless told the input is
    already normalized, type into the rule families."""
    with open(path, "r", encoding="utf-8") as f:
        onto = parse_functional(f.read())
    if not normalized:
        onto = normalize(onto)
    if onto.skipped:
        warnings.warn(f"{path}: axioms without EL+ consequence skipped: {dict(onto.skipped)}")
    return to_axioms(onto)


# ------------------------------------------------------------------ writer
def _fmt(e: Expr) -> str:
    if e[0] == "C":
        return f"<{e[1]}>"
    if e[0] == "I":
        return f"ObjectOneOf(<{e[1]}>)"
    if e[0] == "D":
        return f"<{e[1]}>"
    if e[0] == "AND":
        return "ObjectIntersectionOf(" + " ".join(sorted(_fmt(x) for x in e[1])) + ")"
    if e[0] == "SOME":
        if e[2][0] == "D":
            return f"DataSomeValuesFrom(<{e[1]}> <{e[2][1]}>)"
        return f"ObjectSomeValuesFrom(<{e[1]}> {_fmt(e[2])})"
    raise ValueError(e)


def write_functional(onto: Ontology, path: str) -> int:
    """Save an ontology (e.g. the normalizer's output) in functional syntax, as
    ``Normalizer.normalizeData`` saves ``norm-<file>`` (Normalizer.java:954-959).  Data
    properties used in existentials are declared so the file re-parses identically."""
    lines = []
    for kind, items in (("Class", onto.classes), ("NamedIndividual", onto.individuals),
                        ("ObjectProperty", onto.object_props - onto.data_props),
                        ("DataProperty", onto.data_props), ("Datatype", onto.datatypes)):
        for i in sorted(items):
            lines.append(f"Declaration({kind}(<{i}>))")
    for c, d in onto.sub:
        lines.append(f"SubClassOf({_fmt(c)} {_fmt(d)})")
    for r, s in onto.subrole:
        kw = "SubDataPropertyOf" if r in onto.data_props else "SubObjectPropertyOf"
        lines.append(f"{kw}(<{r}> <{s}>)")
    for chain, s in onto.chain:
        lines.append("SubObjectPropertyOf(ObjectPropertyChain(" + " ".join(f"<{r}>" for r in chain) + f") <{s}>)")
    for r, d in onto.domain:
        kw = "DataPropertyDomain" if r in onto.data_props else "ObjectPropertyDomain"
        lines.append(f"{kw}(<{r}> {_fmt(d)})")
    for r, c in onto.range:
        lines.append(f"ObjectPropertyRange(<{r}> {_fmt(c)})")
    head = f"Ontology(<{onto.iri}>" if onto.iri else "Ontology("
    with open(path, "w", encoding="utf-8") as f:
        f.write(head + "\n" + "\n".join(lines) + "\n)\n")
    return len(lines)


def from_axioms(ax: ir.Axioms, base: str = "urn:distel-amd:ir#") -> Ontology:
    """The ontology an IR stands for (normal forms only), for writing synthetic workloads as
    OWL files.  Names: the IR's concept/role names when they are IRIs, else ``base`` + name."""
    def cname(i: int) -> str:
        if i == ir.BOTTOM:
            return NOTHING
        if i == ir.TOP:
            return THING
        n = ax.concept_name(i)
        return n if ":" in n and not n.startswith("owl:") else base + n

    def rname(i: int) -> str:
        n = ax.role_name(i)
        return n if ":" in n else base + n
    o = Ontology(iri=base.rstrip("#"))
    kinds = ax.kind

    def e(i: int) -> Expr:
        k = int(kinds[i])
        return ("I", cname(i)) if k == ir.KIND_INDIVIDUAL else ("D", cname(i)) if k == ir.KIND_DATATYPE else \
            ("C", cname(i))
    for i in range(2, ax.n_concepts):
        {ir.KIND_CLASS: o.classes, ir.KIND_INDIVIDUAL: o.individuals,
         ir.KIND_DATATYPE: o.datatypes}[int(kinds[i])].add(cname(i))
    o.object_props = {rname(r) for r in range(ax.n_roles)}
    for a, b in ax.sub.tolist():
        o.sub.append((e(a), e(b)))
    for i in range(ax.n_conj):
        ops = frozenset(e(j) for j in ax.conj_ops[ax.conj_ptr[i]:ax.conj_ptr[i + 1]].tolist())
        o.sub.append((("AND", ops) if len(ops) > 1 else next(iter(ops)), e(int(ax.conj_b[i]))))
    for a, r, b in ax.ex_rhs.tolist():
        o.sub.append((e(a), ("SOME", rname(r), e(b))))
    for r, a, b in ax.ex_lhs.tolist():
        o.sub.append((("SOME", rname(r), e(a)), e(b)))
    o.subrole = [(rname(r), rname(s)) for r, s in ax.subrole.tolist()]
    o.chain = [((rname(r), rname(s)), rname(t)) for r, s, t in ax.chain.tolist()]
    o.domain = [(rname(r), e(d)) for r, d in ax.domain.tolist()]
    o.range = [(rname(r), e(c)) for r, c in ax.range.tolist()]
    return o
