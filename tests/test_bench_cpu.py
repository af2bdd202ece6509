"""bench.py's child-process guard: every one-GPU
secondary leg runs in a child under a timeout, so a hung leg is killed and
reported and the headline line still prints.  CPU only: the guard itself."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_child_results_and_exit_code():
    ok, res, _ = bench._child([sys.executable, "-c", "print('{\"a\": 1}'); print('noise'); print('{\"b\": 2}')"],
                              dict(os.environ), 30, "t")
    assert ok and res == [{"a": 1}, {"b": 2}]
    ok, res, err = bench._child([sys.executable, "-c", "import sys; print('{\"a\": 1}'); sys.exit(3)"],
                                dict(os.environ), 30, "t")
    assert not ok and res == [{"a": 1}]


def test_child_killed_at_timeout_keeps_finished_results():
    t0 = time.time()
    ok, res, err = bench._child([sys.executable, "-c",
                                 "import time; print('{\"first\": 1}', flush=True); time.sleep(120)"],
                                dict(os.environ), 3, "t")
    assert time.time() - t0 < 30
    assert not ok and res == [{"first": 1}] and "killed" in err


def test_launch_sets_name_the_traced_kernels():
    """the learner roofline names the kernels rocprofv3 reports for each of
    the reference-order tick's launch sets"""
    f = bench._launch_sets("fp32", "param_noise")
    assert f["acting"].startswith("k_act_step32<true>")
    assert "k_grad_slice_bwd<1>" in f["critic_step"] and "k_grad_slice_bwd<2>" in f["actor_step"]
    assert bench._launch_sets("fp32", "action_noise")["acting"].startswith("k_act_step32<false>")
    assert "k_critic_grad<true>" in bench._launch_sets("bf16", "param_noise")["critic_step"]
