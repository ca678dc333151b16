"""The synthetic graphs of BASELINE.json's configs, generated on the GPU.

One definition serves bench.py (the timed workload) and the headline parity tests, so the
graph a test checks against the oracle is byte for byte the graph the bench line is quoted on.

    configs[0]  R-MAT scale-20, edge factor 16, seed 1          generate("rmat", scale=20)
    configs[1]  LiveJournal-shaped Chung-Lu, seed 4              generate("lj")
    configs[2]  Erdos-Renyi scale-24, degree 16, seed 3          generate("er", scale=24)
    configs[3]  R-MAT scale-26, edge factor 16, seed 2           generate("rmat", scale=26)
    configs[4]  Twitter-2010-shaped Chung-Lu, seed 5             generate("twitter")

Device arrays are torch tensors (PyTorch is only the allocator here); the edges are interned in
first-appearance order on the device (pr_intern_device), as the host interner would.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

from .graph import CHUNGLU_PRESETS, gen_chunglu, gen_er, gen_rmat, intern_device


@dataclass
class Workload:
    src: object  # torch.int32 device tensor of interned source IDs
    dst: object  # torch.int32 device tensor of interned target IDs (-1: record without links)
    n_edges: int  # raw edges (with duplicates and link-less records)
    n_vertices: int
    description: str
    seed: int


def default_seed(graph: str, scale: int) -> int:
    if graph == "rmat":
        return 1 if scale <= 20 else 2
    if graph == "er":
        return 3
    return CHUNGLU_PRESETS[graph]["seed"]


def generate(graph: str, *, scale: int = 26, edge_factor: int = 16, seed: Optional[int] = None,
             device: int = 0) -> Workload:
    import torch

    seed = default_seed(graph, scale) if seed is None else seed
    if graph in ("rmat", "er"):
        E = edge_factor << scale
        labels = 1 << scale
    elif graph in CHUNGLU_PRESETS:
        pre = CHUNGLU_PRESETS[graph]
        E = pre["n_edges"] + pre["n_nolink"]
        labels = pre["n_labels"]
    else:
        raise ValueError(f"unknown graph {graph!r}")
    s = torch.empty(E, dtype=torch.int32, device=f"cuda:{device}")
    d = torch.empty(E, dtype=torch.int32, device=f"cuda:{device}")
    if graph == "rmat":
        gen_rmat(device, scale, E, s.data_ptr(), d.data_ptr(), seed=seed)
        desc = f"R-MAT scale-{scale} edge-factor {edge_factor} (Graph500 .57/.19/.19, seed {seed})"
    elif graph == "er":
        gen_er(device, scale, E, s.data_ptr(), d.data_ptr(), seed=seed)
        desc = f"Erdos-Renyi scale-{scale} degree {edge_factor} (seed {seed})"
    else:
        pre = CHUNGLU_PRESETS[graph]
        gen_chunglu(device, pre["n_labels"], pre["n_edges"], s.data_ptr(), d.data_ptr(), gamma_out=pre["gamma_out"],
                    v0_out=pre["v0_out"], gamma_in=pre["gamma_in"], v0_in=pre["v0_in"], src_frac=pre["src_frac"],
                    n_nolink=pre["n_nolink"], seed=seed)
        desc = (f"{'LiveJournal' if graph == 'lj' else 'Twitter-2010'}-shaped Chung-Lu "
                f"({pre['n_labels']} labels, {pre['n_edges']} edges + {pre['n_nolink']} link-less records, "
                f"gamma out/in {pre['gamma_out']}/{pre['gamma_in']}, seed {seed})")
    V = intern_device(device, E, labels, s.data_ptr(), d.data_ptr())
    return Workload(s, d, E, V, desc, seed)
