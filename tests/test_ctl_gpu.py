"""The reference's custom training loop (tf.GradientTape + apply_gradients,
TFC/core/tests/testdata/mnist_example_using_ctl.py:124-129,150-157) on the NATIVE path of one
MI355X: from step 2 on the variables live in the fused optimizer's arenas and the native
Dense / Conv2D backward writes their gradients there in place -- the tape must return those
gradients (round-4 verdict: it returned zeros and apply_gradients then wiped the arena).

Each check compares final weights after 6 Adam steps on one fixed batch, as the error relative
to how far training moved the weights (zeroed gradients after step 1 leave most of the update
wrong), against: plain autograd + torch.optim.Adam on fp32 masters (native kernels, no arena),
the stock-op path (CLOUD_AMD_OPS=torch), and -- for two replicas sharing the GPU over gloo --
one process over the whole global batch."""
import pytest

from _ctl_util import load, rel_to_update, run_probe

pytestmark = pytest.mark.gpu

GPU = {}
TOL = 0.05  # bf16 compute: rounding differences only


@pytest.fixture(scope="module")
def native_runs(tmp_path_factory):
    d = tmp_path_factory.mktemp("ctl")
    run_probe(d / "ref.npz", env_extra=GPU, args=("--mode", "reference", "--steps", "6"))
    run_probe(d / "ctl.npz", env_extra=GPU, args=("--steps", "6"))
    return d


def test_ctl_native_matches_autograd_reference(native_runs):
    ref, ctl = load(native_runs / "ref.npz"), load(native_runs / "ctl.npz")
    err = rel_to_update(ctl, ref)
    assert err < TOL, (err, ctl[2], ref[2])
    assert ctl[2][-1] < ctl[2][0] and abs(ctl[2][-1] - ref[2][-1]) < 0.02 * abs(ref[2][0])


def test_ctl_native_matches_stock_ops(native_runs, tmp_path):
    run_probe(tmp_path / "torch.npz", env_extra=dict(GPU, CLOUD_AMD_OPS="torch"), args=("--steps", "6"))
    ctl, stock = load(native_runs / "ctl.npz"), load(tmp_path / "torch.npz")
    err = rel_to_update(ctl, stock)
    assert err < TOL, (err, ctl[2], stock[2])


@pytest.mark.timeout(300)
def test_ctl_two_replicas_share_the_gpu_equal_one_process(native_runs, tmp_path):
    out = run_probe(tmp_path / "two.npz", world=2, args=("--steps", "6"),
                    env_extra=dict(GPU, CLOUD_AMD_SHARED_GPU="1", CLOUD_AMD_DIST_BACKEND="gloo"))
    assert out.count("world=2") == 2, out
    one, two = load(native_runs / "ctl.npz"), load(tmp_path / "two.npz")
    err = rel_to_update(two, one)
    assert err < TOL, (err, two[2], one[2])
    assert two[2][-1] < two[2][0]


def test_ctl_loop_makes_no_device_allocations_after_warmup(tmp_path):
    """The run-ahead bound is a property of the fused optimizer's step(): a custom loop with no
    host sync of its own still never grows the caching allocator's pool after warmup."""
    out = run_probe(tmp_path / "a.npz", env_extra=GPU, args=("--steps", "60", "--alloc-warmup", "10"))
    line = [ln for ln in out.splitlines() if ln.startswith("RESULT ctl_alloc")][-1]
    vals = dict(kv.split("=") for kv in line.split()[2:])
    assert int(vals["dev_alloc_after_warmup"]) == 0, line
    assert vals["depth"] != "None", line
