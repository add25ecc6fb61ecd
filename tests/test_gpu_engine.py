"""Single-GPU sessions through the RCCL engine's staging + verification path.

(Multi-rank RCCL transfers need one GPU per rank; those paths are exercised by
the planner/executor tests on CPU and by bench.py on an 8-GPU node.)
"""

import pytest

from distributed_llm_dissemination_amd.models.catalog import make_workload
from distributed_llm_dissemination_amd.parallel.runtime import Runtime, layer_seed

pytestmark = pytest.mark.gpu

MiB = 1 << 20


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_host_tier_promotion_all_modes(gpu, mode):
    cfg = make_workload(1, 6, 6 * MiB + 4096, tier="host", chunk_bytes=MiB)
    rt = Runtime(cfg, 0, engine="rccl", chunk_bytes=MiB, registry={0: "127.0.0.1:0"})
    try:
        for _ in range(2):  # sessions are repeatable (state reset + poison in between)
            res = rt.run(mode, timeout=60)
            assert res.ok, res.error
            assert res.engine_stats["verify_failures"] == 0
            # every staged byte checked exactly once, in every mode (mode 3's
            # self-jobs included): the same count the sim backend gives
            assert res.engine_stats["bytes_staged"] == 6 * (6 * MiB + 4096)
            assert res.engine_stats["bytes_verified"] == 6 * (6 * MiB + 4096)
            for l in range(6):
                assert rt.layer_bytes(l) == gpu.fill_random_host(6 * MiB + 4096, layer_seed(0, l))
    finally:
        rt.close()


@pytest.mark.parametrize("mode", [0, 1])
def test_layer_size_not_a_multiple_of_16(gpu, mode):
    """Layers of any byte size (the reference's experiment layers are 10,930,691,768 B):
    the last chunk of every layer has a length that is not a multiple of 16."""
    size = 3 * MiB + 13
    cfg = make_workload(1, 3, size, tier="host", chunk_bytes=MiB)
    rt = Runtime(cfg, 0, engine="rccl", chunk_bytes=MiB, registry={0: "127.0.0.1:0"})
    try:
        res = rt.run(mode, timeout=60)
        assert res.ok, res.error
        assert res.engine_stats["verify_failures"] == 0
        for l in range(3):
            assert rt.layer_bytes(l) == gpu.fill_random_host(size, layer_seed(0, l))
    finally:
        rt.close()


def test_device_seeded_nothing_to_move(gpu):
    cfg = make_workload(1, 3, 2 * MiB, tier="device", chunk_bytes=MiB)
    rt = Runtime(cfg, 0, engine="rccl", chunk_bytes=MiB, registry={0: "127.0.0.1:0"})
    try:
        res = rt.run(1, timeout=30)
        assert res.ok and res.bytes_planned == 0
    finally:
        rt.close()


def test_corrupt_manifest_is_detected(gpu):
    cfg = make_workload(1, 2, 2 * MiB, tier="host", chunk_bytes=MiB)
    rt = Runtime(cfg, 0, engine="rccl", chunk_bytes=MiB, registry={0: "127.0.0.1:0"})
    try:
        bad = gpu.CrcManifest(MiB, [0xDEADBEEF, 0x12345678])
        rt.engine.set_manifest(1, bad)
        res = rt.run(1, timeout=10)
        assert not res.ok
        assert "CRC32C mismatch" in res.error
    finally:
        rt.close()


def test_gpu_topology_probe(gpu):
    import torch

    n = torch.cuda.device_count()
    topo = gpu.gpu_topology()
    assert len(topo) == n * (n - 1)
    for i, j, kind, hops, p2p in topo:
        assert i != j and kind in ("xgmi", "pcie", "other") and hops >= 0
    if n > 1:  # an MI355X node: fully connected xGMI
        assert all(kind == "xgmi" and p2p for _, _, kind, _, p2p in topo)


@pytest.mark.parametrize("tier", ["host", "device", "disk"])
def test_fp8_packed_session(gpu, tier, tmp_path):
    """--pack fp8 on one GPU: bf16 sources are packed on the copy stream while
    staging; the HBM slot holds the packed image the manifest was computed on,
    and the fused verify+unpack kernel restores the bf16 layer."""
    size = 3 * MiB + 4096
    cfg = make_workload(1, 3, size, tier=tier, chunk_bytes=MiB)
    rt = Runtime(cfg, 0, engine="rccl", chunk_bytes=MiB, registry={0: "127.0.0.1:0"}, pack="fp8",
                 storage_path=str(tmp_path) if tier == "disk" else "")
    try:
        images = {l: rt.layer_bytes(l) for l in range(3)}  # after materialize: the packed image
        for _ in range(2):
            res = rt.run(1, timeout=60)
            assert res.ok, res.error
            assert res.engine_stats["verify_failures"] == 0
            for l in range(3):
                assert rt.layer_bytes(l) == images[l]
                out = rt.unpacked_layer_bytes(l)
                assert out == gpu.fp8_unpack_layer_host(images[l], size, MiB, 128)
    finally:
        rt.close()


def test_hbm_capacity_is_checked_before_allocating():
    """A placement larger than the GPU's HBM is refused up front with a clear
    message (no partial allocation): 80 x 4 GiB = 320 GiB > 288 GB."""
    from distributed_llm_dissemination_amd.models.catalog import make_workload
    from distributed_llm_dissemination_amd.parallel.runtime import Runtime

    cfg = make_workload(1, 80, 4 << 30, tier="device", chunk_bytes=64 << 20)
    with pytest.raises(ValueError, match="HBM"):
        Runtime(cfg, 0, engine="rccl", chunk_bytes=64 << 20, registry={0: "127.0.0.1:0"})


@pytest.mark.parametrize("pack", ["none", "fp8"])
def test_layer_weights_zero_copy_in_hbm(gpu, pack):
    """A Llama-family decoder layer (models/weights.py) staged into HBM by a session,
    read back as named bf16 parameters that alias the HBM slot (or, with fp8, the
    dequantized image the fused verify+unpack wrote) and run on the GPU."""
    import torch

    from distributed_llm_dissemination_amd.models.weights import (PRESETS, decoder_forward, flatten, layer_nbytes,
                                                                 random_layer, unflatten)

    spec = PRESETS["tiny"]
    size = layer_nbytes(spec)
    blobs = {l: flatten(random_layer(spec, 7 + l), spec) for l in range(2)}
    cfg = make_workload(1, 2, size, tier="host", chunk_bytes=64 * 1024)
    rt = Runtime(cfg, 0, engine="rccl", chunk_bytes=64 * 1024, registry={0: "127.0.0.1:0"}, pack=pack,
                 store="bf16" if pack == "fp8" else "packed", layer_source=lambda l, n: blobs[l])
    try:
        res = rt.run(1, timeout=60)
        assert res.ok, res.error
        x = torch.randn(1, 16, spec.hidden).to(torch.bfloat16)
        for l in range(2):
            p = rt.layer_params(l, spec)
            t = rt.layer_tensor(l, unpacked=True)
            assert t.is_cuda and t.numel() == size
            want_ptr = rt.engine.unpacked_ptr(l) if pack == "fp8" else rt.engine.device_ptr(l)
            assert t.data_ptr() == want_ptr and p["input_layernorm"].data_ptr() == want_ptr  # zero-copy
            want = unflatten(blobs[l], spec)
            if pack == "none":
                assert all(torch.equal(p[k].cpu(), want[k]) for k in want)
            else:
                ref = gpu.fp8_unpack_layer_host(gpu.fp8_pack_layer_host(blobs[l].numpy().tobytes(), 64 * 1024, 128),
                                                size, 64 * 1024, 128)
                assert t.cpu().numpy().tobytes() == ref
            y = decoder_forward(x.cuda(), p, spec).float().cpu()
            y0 = decoder_forward(x, {k: p[k].cpu() for k in p}, spec).float()
            assert float((y - y0).norm() / y0.norm()) < 2e-2
    finally:
        rt.close()


@pytest.mark.parametrize("verify_cus,store", [(32, "packed"), (128, "bf16")])
def test_verify_on_its_own_cus(gpu, verify_cus, store):
    """The verify stream on the last `verify_cus` CUs, copies (and RCCL lanes) on the
    others (hip_backend.h verify_cus: the default with peers): every chunk still
    verified; with the fused fp8 unpack the check and the unpack share those CUs."""
    size = 6 * MiB + 4096
    kw = {"pack": "fp8", "store": "bf16"} if store == "bf16" else {}
    cfg = make_workload(1, 6, size, tier="host", chunk_bytes=MiB)
    rt = Runtime(cfg, 0, engine="rccl", chunk_bytes=MiB, registry={0: "127.0.0.1:0"},
                 engine_opts={"verify_cus": verify_cus}, **kw)
    try:
        res = rt.run(1, timeout=60)
        assert res.ok, res.error
        assert res.engine_stats["verify_failures"] == 0
        for l in range(6):
            if store == "packed":
                assert rt.layer_bytes(l) == gpu.fill_random_host(size, layer_seed(0, l))
            else:  # the fused check + unpack on the verify CUs restored the bf16 layer
                assert rt.unpacked_layer_bytes(l) == gpu.fp8_unpack_layer_host(rt.layer_bytes(l), size, MiB, 128)
    finally:
        rt.close()
