"""Device argument tables and the lifetime of the buffers they point at.

Grouped launches read their operands through device tables: ctypes struct arrays of raw device
pointers (hv_kernels.h) uploaded once and replayed many times (prep programs, the grouped
training prep, Sinkhorn groups, NMS plans, the optimizer table, captured graphs).  A raw pointer
keeps nothing alive: a buffer referenced ONLY by a table is released by the caching allocator,
reused, and the next replay writes into someone else's memory (round 5 hit this twice:
`k_pg4` wrote into a freed row-sum buffer, and a graph's prep program outlived its owner).

The rule every table builder follows: each pointer it writes lies inside a tensor the OWNING
program itself holds (an attribute, a list/dict/dataclass inside it, or a parameter / buffer of
a module it holds).  `upload(entries, device, owner, name)` records the table on its owner, and
`unheld_pointers(owner)` walks every recorded table and returns the pointers no held tensor
covers -- run by the CPU suite on programs built from CPU tensors (tests/test_tables_cpu.py) and
by the GPU suite on the live programs of a forward and a training step.
"""
from __future__ import annotations

import ctypes as C
import dataclasses
from typing import Dict, Iterator, List, Tuple

import torch
import torch.nn as nn

_TABLES = "_hv_tables"


def register(owner, name: str, entries) -> None:
    """Record `entries` (a ctypes struct array) as owner's table `name` (replacing an older one
    of the same name: a rebuilt table supersedes it)."""
    owner.__dict__.setdefault(_TABLES, {})[name] = entries


def upload(entries, device, owner, name: str) -> torch.Tensor:
    """register() + the asynchronous upload of ops.upload_table."""
    from .ops import upload_bytes
    register(owner, name, entries)
    return upload_bytes(bytes(entries), device)


def _pointer_fields(struct, prefix: str = "") -> Iterator[Tuple[str, int]]:
    for fname, ftype in struct._fields_:
        v = getattr(struct, fname)
        if ftype is C.c_void_p:
            if v:
                yield prefix + fname, int(v)
        elif isinstance(ftype, type) and issubclass(ftype, C.Structure):
            yield from _pointer_fields(v, prefix + fname + ".")


def table_pointers(entries) -> Iterator[Tuple[int, str, int]]:
    """(entry index, field, pointer) for every non-null pointer field of a struct array."""
    for i in range(len(entries)):
        for f, p in _pointer_fields(entries[i]):
            yield i, f, p


def _storage_span(t: torch.Tensor) -> Tuple[int, int]:
    s = t.untyped_storage()
    return s.data_ptr(), s.data_ptr() + s.nbytes()


def held_spans(owner) -> List[Tuple[int, int]]:
    """[start, end) byte spans of every tensor storage reachable from `owner`: its attributes,
    containers and dataclasses inside them, objects of this package, and the parameters, their
    gradients and the buffers of any module held."""
    spans: List[Tuple[int, int]] = []
    seen = set()
    stack = [owner]
    while stack:
        o = stack.pop()
        if id(o) in seen or o is None:
            continue
        seen.add(id(o))
        if isinstance(o, torch.Tensor):
            if o.device.type != "meta" and o.untyped_storage().nbytes():
                spans.append(_storage_span(o))
            if o.is_leaf and o.grad is not None:
                stack.append(o.grad)
        elif isinstance(o, nn.Module):
            stack.extend(o.parameters())
            stack.extend(o.buffers())
        elif isinstance(o, dict):
            stack.extend(v for k, v in o.items() if k != _TABLES)
        elif isinstance(o, (list, tuple, set, frozenset)):
            stack.extend(o)
        elif dataclasses.is_dataclass(o) and not isinstance(o, type):
            stack.extend(getattr(o, f.name) for f in dataclasses.fields(o))
        elif type(o).__module__.startswith("hv_amd") and hasattr(o, "__dict__"):
            stack.extend(v for k, v in vars(o).items() if k != _TABLES)
    return spans


def unheld_pointers(owner) -> List[Tuple[str, int, str, int]]:
    """(table, entry, field, pointer) of every recorded table pointer that no tensor held by
    `owner` covers.  Empty = the program keeps alive everything its tables point at."""
    tables: Dict[str, object] = owner.__dict__.get(_TABLES, {})
    spans = sorted(held_spans(owner))
    bad = []
    for name, entries in tables.items():
        for i, f, p in table_pointers(entries):
            if not any(a <= p < b for a, b in spans):
                bad.append((name, i, f, p))
    return bad
