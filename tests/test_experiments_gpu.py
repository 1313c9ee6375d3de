"""The kernel arms kept for the record in tools/experiments/libexperiments.so
(not the product): each must still equal the oracle, so the numbers in
profiles/ and DESIGN.md section 4 stay reproducible.  One pass over the golden
images and one corrupted Zipf image per arm; the production paths get the
full parity suite in test_gpu.py."""
import numpy as np
import pytest

import test_gpu
from conftest import golden_image
from oracle import oracle_c as oc
from test_gpu import BLOCK_SIZE, compare_walk, kat_blocks, run_full, zipf_image

# Not part of the driver's `-m gpu` product suite: run with `-m experiment` on
# a GPU box after `make -C tools/experiments` (conftest skips them otherwise).
pytestmark = pytest.mark.experiment

C3_ARMS = [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 20, 21, 22, 23, 24, 30]
C2_ARMS = [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 20, 21, 22]  # 100-106: read-ceiling shapes, no CRC


@pytest.mark.parametrize("variant", C3_ARMS)
def test_c3_verify_arm_vs_oracle(gpu_ctx, golden_index, variant):
    for name in golden_index:
        img = golden_image(name)
        dimg = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
        compare_walk(gpu_ctx.verify_image(dimg, len(img), variant=variant), oc.walk(img))
    rng = np.random.default_rng(13)
    img = bytearray(oc.write_image(zipf_image(rng, 4 << 20)))
    ref = oc.walk(bytes(img))
    for v in rng.choice(np.flatnonzero(ref["length"] > 0), 30, replace=False):
        img[int(ref["file_offset"][v]) + 7 + int(rng.integers(0, int(ref["length"][v])))] ^= 4
    img = bytes(img)
    dimg = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
    compare_walk(gpu_ctx.verify_image(dimg, len(img), variant=variant), oc.walk(img))


@pytest.mark.parametrize("variant", C2_ARMS)
def test_c2_crc_arm_vs_oracle(gpu_ctx, variant):
    blocks = kat_blocks()
    rng = np.random.default_rng(variant)
    extra = rng.integers(0, 256, (300, blocks.shape[1]), dtype=np.uint8)
    extra[:, 4], extra[:, 5], extra[:, 6] = 0xF9, 0x7F, 1
    blocks = np.vstack([blocks, extra])
    got, _ = run_full(gpu_ctx, blocks, variant=variant)
    assert np.array_equal(got, oc.full_block_crcs(blocks))


def walk_verify(gpu_ctx, dimg, n):
    """The fused pipeline (x_verify_walk.inc): revel_x_walk_count_scan ->
    revel_x_walk_verify, results as verify_image's."""
    from revel_amd._lib import check, experiments
    from revel_amd.gpu import RECORD_DTYPE
    X = experiments()
    nblocks = (n + 32767) // 32768
    counts, first = gpu_ctx.alloc(4 * nblocks), gpu_ctx.alloc(4 * nblocks)
    check(X.revel_x_walk_count_scan(gpu_ctx.handle, dimg.ptr, n, counts.ptr, first.ptr, None))
    total = int(gpu_ctx.d2h(first, 4, np.uint32, src_offset=4 * (nblocks - 1))[0]) + \
        int(gpu_ctx.d2h(counts, 4, np.uint32, src_offset=4 * (nblocks - 1))[0])
    out = gpu_ctx.alloc(max(1, total) * RECORD_DTYPE.itemsize)
    check(X.revel_x_walk_verify(gpu_ctx.handle, dimg.ptr, n, 0, counts.ptr, first.ptr, out.ptr, None))
    gpu_ctx.sync()
    return gpu_ctx.d2h(out, total * RECORD_DTYPE.itemsize, np.uint8).view(RECORD_DTYPE)


def test_walk_pipeline_vs_oracle(gpu_ctx, golden_index):
    """The fused pipeline (measured slower than the count pass, kept as an
    experiment): golden images, a corrupted Zipf image, dense blocks with
    records past kListCap, 32-word record streams, a partial tail block."""
    images = [golden_image(name) for name in golden_index]
    rng = np.random.default_rng(17)
    img = bytearray(oc.write_image(zipf_image(rng, 4 << 20)))
    ref = oc.walk(bytes(img))
    for v in rng.choice(np.flatnonzero(ref["length"] > 0), 30, replace=False):
        img[int(ref["file_offset"][v]) + 7 + int(rng.integers(0, int(ref["length"][v])))] ^= 4
    images.append(bytes(img))
    images.append(oc.write_image([rng.integers(0, 256, int(s), dtype=np.uint8).tobytes()
                                  for s in rng.integers(0, 40, 20000)]))
    images.append(oc.write_image([bytes(127) for _ in range(700)]))
    images.append(oc.write_image([bytes(64 * 64 + 9) for _ in range(70)])[:-5000])
    for img in images:
        dimg = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
        compare_walk(walk_verify(gpu_ctx, dimg, len(img)), oc.walk(img))


# ---- round 5's small-record kernels (moved out of the product in round 6) ----
# "one_pass" / "one_pass2": the one-pass count + checksum pair
# (revel_x_fused_count_scan mode 1 / 2 -> revel_x_fused_verify);
# "dense_chunks" / "dense_quad" / "dense_sorted": the production split with
# k_verify_dense_chunks, dense2's quad-coalesced loads or round 6's
# length-sorted batches for the dense blocks (revel_x_verify_dense_variant);
# "dense_staged*": round 6's batch spans staged in LDS (8 or 12 waves per CU,
# 2 or 1 chains per lane, x_verify_dense_staged.inc).  Every verify test of
# test_gpu.py that the product runs over its VERIFY_PATHS runs here over these.
STAGED_PATHS = ["dense_staged", "dense_staged_1ch", "dense_staged_12w", "dense_staged_12w_1ch", "dense_staged_a16",
                "dense_staged_a16_8w"]
EXPERIMENT_PATHS = ["one_pass", "one_pass2", "dense_chunks", "dense_quad", "dense_sorted", "dense_pairs"] + STAGED_PATHS


@pytest.fixture
def experiment_paths(monkeypatch):
    monkeypatch.setattr(test_gpu, "VERIFY_PATHS", EXPERIMENT_PATHS)


@pytest.mark.parametrize("path", EXPERIMENT_PATHS)
def test_exp_verify_golden_images(gpu_ctx, golden_index, path):
    test_gpu.test_verify_golden_images(gpu_ctx, golden_index, path)


@pytest.mark.parametrize("path", EXPERIMENT_PATHS)
def test_exp_verify_zipf_and_corruption(gpu_ctx, path):
    test_gpu.test_verify_zipf_and_corruption(gpu_ctx, path)


@pytest.mark.parametrize("path", EXPERIMENT_PATHS)
@pytest.mark.parametrize("cut", [1, 3, 6, 7, 8, 100, 32767, 32769, 40000])
def test_exp_verify_partial_last_block(gpu_ctx, cut, path):
    test_gpu.test_verify_partial_last_block(gpu_ctx, cut, path)


def test_exp_loop_tests(gpu_ctx, experiment_paths):
    """The product's loop-over-VERIFY_PATHS tests with the experiment paths."""
    test_gpu.test_full_blocks_large_property(gpu_ctx)
    test_gpu.test_expander_counts_1_to_64_with_flips(gpu_ctx)
    for plen in [123, 124, 126, 127, 128, 251, 254, 255, 256]:
        test_gpu.test_verify_dense_word_stream_edges(gpu_ctx, plen)
    test_gpu.test_verify_small_records_dense(gpu_ctx)
    for rec_len in [24, 100, 124, 200]:
        test_gpu.test_verify_multi_batch_lists(gpu_ctx, rec_len)
    test_gpu.test_verify_batch_start_on_16_byte_boundary(gpu_ctx)
    for tail in ["dense", "sparse"]:
        test_gpu.test_verify_mixed_density(gpu_ctx, tail)
    test_gpu.test_property_dense_streams_vs_oracle(gpu_ctx)
    for tail in [1, 3, 7, 11]:
        for slack in [0, 2, 6]:
            test_gpu.test_dense_block_then_tiny_tail(gpu_ctx, tail, slack)
    for seed in [0, 1, 2]:
        test_gpu.test_dense_chunks_markers_and_reuse(gpu_ctx, seed)


@pytest.mark.parametrize("path", EXPERIMENT_PATHS + [None])
@pytest.mark.parametrize("ending", ["zero", "bad_length"])
def test_exp_256_records_then_bad_header(gpu_ctx, path, ending):
    """a block of exactly 256 valid records followed by a
    zero header or a length past the block end.  The one-pass kernels listed
    such a block for dense2 with resume offset 0, so record 256 was re-read
    from record 0's header; the oracle makes record 256 a status record."""
    rng = np.random.default_rng(256)
    n = 256
    body = 32768 - 7 * n - 600  # room left for the bad header in the block
    recs = test_gpu._block_of_records(rng, n, body)
    img = bytearray(oc.write_image(recs))
    off = len(img)  # header of record 256, inside block 0
    assert off + 7 <= 32768
    if ending == "zero":
        img += bytes(7)
    else:
        img += bytes([1, 2, 3, 4]) + (0x7FF0).to_bytes(2, "little") + bytes([1])
    img += bytes(32768 - len(img))  # pad the block
    img = bytes(img)
    ref = oc.walk(img)
    assert len(ref) == n + 1 and ref["status"][n] != 0
    dimg = gpu_ctx.upload(np.frombuffer(img, dtype=np.uint8))
    compare_walk(gpu_ctx.verify_image(dimg, len(img), path=path), ref)


LONG_SHAPES = ["long_last", "long_first", "long_mid_flip", "over_256", "two_long", "tail"]


@pytest.mark.parametrize("path", STAGED_PATHS + ["dense_pairs", None])
@pytest.mark.parametrize("shape", LONG_SHAPES)
def test_exp_dense_blocks_with_long_records(gpu_ctx, path, shape):
    """Dense blocks (more than 64 records) that also hold a record longer
    than a staged batch's LDS slot (8-16 KiB): the staged kernels checksum it
    piece by piece with the whole wave; checked field by field against the
    oracle walk, with flips inside the long records and next to them."""
    rng = np.random.default_rng(LONG_SHAPES.index(shape))
    tiny = lambda k: [rng.integers(0, 256, int(rng.integers(0, 24)), dtype=np.uint8).tobytes() for _ in range(k)]
    big = lambda n: rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    recs = []
    for blk in range(6):
        if shape == "long_last":
            recs += tiny(90) + [big(BLOCK_SIZE - 90 * 20 - 200 - int(rng.integers(0, 300)))]
        elif shape == "long_first":
            recs += [big(20000 + int(rng.integers(0, 5000)))] + tiny(120)
        elif shape == "long_mid_flip":
            recs += tiny(70) + [big(12000 + 997 * blk)] + tiny(100)
        elif shape == "over_256":
            recs += [b""] * 300 + [big(16000 + int(rng.integers(0, 9000)))] + tiny(10)
        elif shape == "two_long":
            recs += tiny(66) + [big(9000 + 13 * blk), big(8190 + 111 * blk)] + tiny(40)
        else:
            recs += tiny(200) + [big(13000)]
    img = bytearray(oc.write_image(recs))
    ref = oc.walk(bytes(img))
    for v in range(3, len(ref), 29):
        if int(ref["length"][v]) > 0:
            off = int(ref["file_offset"][v]) + 7 + int(rng.integers(0, int(ref["length"][v])))
            img[off] ^= 1 << int(rng.integers(0, 8))
    if shape == "tail":
        img = img[:len(img) - 777]  # a partial dense last block
    ref = oc.walk(bytes(img))
    assert (np.bincount(ref["file_offset"] // BLOCK_SIZE) > 64).any()
    dimg = gpu_ctx.upload(np.frombuffer(bytes(img), dtype=np.uint8))
    test_gpu.compare_walk(gpu_ctx.verify_image(dimg, len(img), path=path), ref)
