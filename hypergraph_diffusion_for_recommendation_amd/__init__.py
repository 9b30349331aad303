"""MI355X-native hypergraph propagation for SELFRec-style recommenders.

The hot path — the incidence SpMM hops of HGNN / HCCF / ED-HNN ("hypergraph diffusion")
propagation and their backward — runs in hand-written gfx950 HIP kernels behind the C ABI of
``include/hgd.h`` (``_lib/libhgd.so``). The modules here sequence those calls and expose them
with the reference's operator signatures:

* :mod:`.incidence`  — device CSR/CSC structures (replaces per-call COO coalesce / ``adj.t()``)
* :mod:`.functional` — autograd hops: ``spmm``, ``two_hop``, ``hgconv2``, ``mean2hop``
* :mod:`.layers`     — drop-in ``GCNLayer``, ``HGNNLayer``, ``HGCNConv``, ``SpAdjDropEdge``,
                       ``EquivSetConv``, ``EquivSetGNN``, ``MLP``
* :mod:`.sharded`    — user-row sharding across GPUs with an RCCL all-reduce of hyperedge sums
"""
from . import _native
from .incidence import CSR, Incidence, incidence_of, spmm_csr
from .functional import contrast_loss, hgconv2, mean2hop, spmm, two_hop, unique_long

__all__ = ["CSR", "Incidence", "incidence_of", "spmm_csr", "spmm", "two_hop", "hgconv2",
           "mean2hop", "contrast_loss", "unique_long", "_native"]
__version__ = "0.1.0"
