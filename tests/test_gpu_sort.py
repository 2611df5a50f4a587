"""The engine's stable LSD radix sort (icp_sort.hip, through icp_sort_pairs) against numpy's
stable argsort of the masked keys.

The sort orders the grid build's cell lists (launch_grid_build) and the scene's slot order
(launch_slot_order_aos) -- the orders rounds 4-5 took from rocprim's onesweep sort, which is
stable too, so the order must be exactly (key & mask, input position).  Cases: every digit count
(1-4 passes, odd and even, so both ping-pong ends), partial and exact tiles (4,096 items), keys
with bits above `bits` (ignored), all-equal keys (the identity), sorted and reversed inputs,
a skewed key distribution (one digit holding most of a tile), bits = 0 and n = 0.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def amd(icp_lib):
    if icp_lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    return icp_lib


def expect(keys, bits):
    masked = keys.astype(np.uint64) & ((1 << bits) - 1)
    order = np.argsort(masked, kind="stable").astype(np.int32)
    return order, keys[order]


def check(amd, keys, bits):
    order, out = amd.sort_pairs(keys, bits)
    eo, ek = expect(keys, bits)
    assert np.array_equal(order, eo)
    assert np.array_equal(out, ek)


@pytest.mark.parametrize("n", [1, 100, 4095, 4096, 4097, 3 * 4096 + 17, (1 << 20) + 123])
@pytest.mark.parametrize("bits", [1, 7, 8, 9, 15, 19, 21, 24, 32])
def test_random_keys(amd, n, bits):
    rng = np.random.default_rng(n * 37 + bits)
    keys = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    check(amd, keys, bits)


@pytest.mark.parametrize("bits", [8, 21, 24])
def test_few_distinct_keys(amd, bits):
    """Long runs of equal keys (most grid cells hold a few points; ties decide the cell lists)."""
    rng = np.random.default_rng(bits)
    keys = rng.integers(0, 5, size=200_003).astype(np.uint32) * 4099
    check(amd, keys, bits)


def test_equal_keys_keep_input_order(amd):
    keys = np.full(50_000, 0x00ABCDEF, dtype=np.uint32)
    order, out = amd.sort_pairs(keys, 24)
    assert np.array_equal(order, np.arange(keys.size, dtype=np.int32))
    assert np.array_equal(out, keys)


@pytest.mark.parametrize("form", ["sorted", "reversed", "skewed"])
def test_structured_inputs(amd, form):
    n = 300_000
    rng = np.random.default_rng(3)
    keys = np.sort(rng.integers(0, 1 << 21, size=n)).astype(np.uint32)
    if form == "reversed":
        keys = keys[::-1].copy()
    elif form == "skewed":  # most keys share one value, the rest spread
        keys = np.where(rng.random(n) < 0.9, 777, rng.integers(0, 1 << 21, size=n)).astype(np.uint32)
    check(amd, keys, 21)


def test_bits_zero_and_empty(amd):
    keys = np.arange(1000, 0, -1, dtype=np.uint32)
    order, out = amd.sort_pairs(keys, 0)
    assert np.array_equal(order, np.arange(1000, dtype=np.int32))
    assert np.array_equal(out, keys)
    order, out = amd.sort_pairs(np.empty(0, dtype=np.uint32), 24)
    assert order.size == 0 and out.size == 0


def test_bad_bits_rejected(amd):
    with pytest.raises(amd.ICPError):
        amd.sort_pairs(np.zeros(4, dtype=np.uint32), 33)
