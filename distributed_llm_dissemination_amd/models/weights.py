"""Decoder-layer weights as dissemination layers (the serving side of the service).

The engine moves a layer as opaque bytes (reference semantics: a layer is a
byte blob of ``LayerSize``). A model deployment wants those bytes back as the
layer's named parameters. This module fixes a byte layout for one decoder layer
of a Llama-family model - its parameters in a fixed order, each contiguous, the
blob padded to a 4 KiB multiple (so fp8 packing's whole scale blocks and the
chunk grid both fit) - and converts between the two:

    spec = PRESETS["llama3-70b"]
    blob = flatten(weights, spec)                 # host side: the layer's source bytes
    rt = Runtime(cfg, rank, ..., layer_source=lambda l, n: blobs[l])
    ...session...
    params = rt.layer_params(l, spec)             # named bf16 views of the layer in HBM (zero-copy)
    y = decoder_forward(x, params, spec)          # use them

``decoder_forward`` is a plain PyTorch reference of the layer (RMSNorm,
grouped-query attention with rotary embeddings, SwiGLU MLP) that the tests run
on received weights against the originals.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Tuple

import torch
import torch.nn.functional as F

ALIGN = 4096


@dataclass(frozen=True)
class DecoderSpec:
    name: str
    hidden: int
    intermediate: int
    heads: int
    kv_heads: int
    layers: int
    rope_theta: float = 500000.0
    eps: float = 1e-5

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads


PRESETS: Dict[str, DecoderSpec] = {
    "llama3-8b": DecoderSpec("llama3-8b", 4096, 14336, 32, 8, 32),
    "llama3-70b": DecoderSpec("llama3-70b", 8192, 28672, 64, 8, 80),
    "llama3.1-405b": DecoderSpec("llama3.1-405b", 16384, 53248, 128, 8, 126),
    "tiny": DecoderSpec("tiny", 256, 512, 4, 2, 4),
}


def layer_params(spec: DecoderSpec) -> List[Tuple[str, Tuple[int, ...]]]:
    """(name, shape) of one decoder layer's parameters, in blob order (torch Linear: [out, in])."""
    h, i, kv = spec.hidden, spec.intermediate, spec.kv_heads * spec.head_dim
    return [
        ("input_layernorm", (h,)),
        ("q_proj", (h, h)),
        ("k_proj", (kv, h)),
        ("v_proj", (kv, h)),
        ("o_proj", (h, h)),
        ("post_attention_layernorm", (h,)),
        ("gate_proj", (i, h)),
        ("up_proj", (i, h)),
        ("down_proj", (h, i)),
    ]


def _numel(shape) -> int:
    n = 1
    for s in shape:
        n *= s
    return n


def layer_nbytes(spec: DecoderSpec, elem_bytes: int = 2) -> int:
    """Bytes of one layer's blob (bf16 parameters, padded to ALIGN)."""
    raw = sum(_numel(s) for _, s in layer_params(spec)) * elem_bytes
    return -(-raw // ALIGN) * ALIGN


def random_layer(spec: DecoderSpec, seed: int, dtype=torch.bfloat16) -> Dict[str, torch.Tensor]:
    """Initialised like a real layer (norm weights 1 +- noise, projections ~N(0, 1/fan_in))."""
    g = torch.Generator().manual_seed(seed)
    out = {}
    for name, shape in layer_params(spec):
        if len(shape) == 1:
            w = 1.0 + 0.02 * torch.randn(shape, generator=g)
        else:
            w = torch.randn(shape, generator=g) / shape[1] ** 0.5
        out[name] = w.to(dtype)
    return out


def flatten(weights: Dict[str, torch.Tensor], spec: DecoderSpec) -> torch.Tensor:
    """The layer's blob: a contiguous uint8 CPU tensor of layer_nbytes(spec) bytes."""
    blob = torch.zeros(layer_nbytes(spec), dtype=torch.uint8)
    off = 0
    for name, shape in layer_params(spec):
        w = weights[name]
        if tuple(w.shape) != shape or w.dtype != torch.bfloat16:
            raise ValueError(f"{name}: expected bf16 {shape}, got {w.dtype} {tuple(w.shape)}")
        n = w.numel() * 2
        blob[off:off + n] = w.detach().cpu().contiguous().view(-1).view(torch.uint8)
        off += n
    return blob


def unflatten(blob: torch.Tensor, spec: DecoderSpec) -> Dict[str, torch.Tensor]:
    """Named bf16 views of a layer blob (uint8 or bf16 tensor on any device; no copy)."""
    if blob.dtype != torch.uint8:
        blob = blob.view(torch.uint8)
    blob = blob.view(-1)
    if blob.numel() < layer_nbytes(spec):
        raise ValueError(f"blob holds {blob.numel()} B, the layer needs {layer_nbytes(spec)}")
    out = {}
    off = 0
    for name, shape in layer_params(spec):
        n = _numel(shape) * 2
        out[name] = blob[off:off + n].view(torch.bfloat16).view(shape)
        off += n
    return out


def _rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()).to(x.dtype)


def _rope(x: torch.Tensor, theta: float) -> torch.Tensor:
    """Rotary embedding over [batch, heads, seq, head_dim] (rotate-half convention)."""
    d = x.shape[-1]
    inv = 1.0 / (theta ** (torch.arange(0, d, 2, device=x.device, dtype=torch.float32) / d))
    pos = torch.arange(x.shape[-2], device=x.device, dtype=torch.float32)
    ang = torch.outer(pos, inv)
    cos, sin = torch.cat([ang, ang], -1).cos(), torch.cat([ang, ang], -1).sin()
    x1, x2 = x.float()[..., : d // 2], x.float()[..., d // 2:]
    return (x.float() * cos + torch.cat([-x2, x1], -1) * sin).to(x.dtype)


def decoder_forward(x: torch.Tensor, p: Dict[str, torch.Tensor], spec: DecoderSpec) -> torch.Tensor:
    """One decoder layer on x [batch, seq, hidden] (causal self-attention, no KV cache)."""
    b, s, _ = x.shape
    hd, nh, nkv = spec.head_dim, spec.heads, spec.kv_heads
    h = _rms_norm(x, p["input_layernorm"], spec.eps)
    q = F.linear(h, p["q_proj"]).view(b, s, nh, hd).transpose(1, 2)
    k = F.linear(h, p["k_proj"]).view(b, s, nkv, hd).transpose(1, 2)
    v = F.linear(h, p["v_proj"]).view(b, s, nkv, hd).transpose(1, 2)
    q, k = _rope(q, spec.rope_theta), _rope(k, spec.rope_theta)
    k = k.repeat_interleave(nh // nkv, dim=1)
    v = v.repeat_interleave(nh // nkv, dim=1)
    a = F.scaled_dot_product_attention(q, k, v, is_causal=True)
    x = x + F.linear(a.transpose(1, 2).reshape(b, s, nh * hd), p["o_proj"])
    h = _rms_norm(x, p["post_attention_layernorm"], spec.eps)
    return x + F.linear(F.silu(F.linear(h, p["gate_proj"])) * F.linear(h, p["up_proj"]), p["down_proj"])
