"""MI355X-native LLM layer dissemination.

A leader rank and N receiver ranks place LLM weight shards ("layers") into the
HBM of every GPU that an Assignment names, using one of four distribution
modes (0 naive, 1 retransmit, 2 pull/steal, 3 max-flow) with the same CLI and
JSON config as ynishimi/distributed-llm-dissemination (reference).

Layout:
  _core            native runtime (C++ roles/transports/schedulers + HIP kernels + RCCL engine)
  utils/           config schema, JSONL logs, launch helpers
  parallel/        rank bootstrap, data-plane selection, session runner
  ops/             Python wrappers of the gfx950 kernels (fill, CRC32C, fp8 pack)
  models/          layer catalogs of real models (Llama-3-70B / 405B shard sizes)
"""

# torch first: _core links the HIP runtime and RCCL shipped with PyTorch-ROCm,
# so importing torch first guarantees one copy of each in the process.
import torch  # noqa: F401

from . import _core  # noqa: E402
from ._core import (  # noqa: E402,F401
    CLIENT_ID,
    LayerMeta,
    LayerSrc,
    Location,
    Message,
    MsgType,
    Node,
    NodeConfig,
    SourceType,
)

__all__ = [
    "_core",
    "CLIENT_ID",
    "LayerMeta",
    "LayerSrc",
    "Location",
    "Message",
    "MsgType",
    "Node",
    "NodeConfig",
    "SourceType",
]
__version__ = "0.1.0"
