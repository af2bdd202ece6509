"""F4 on-disk formats (SkillshotLearner.py:123-204 layout; persist.py states
the deliberate differences): models round-trip through safetensors with the
reference's epoch-range names, the progress CSV appends, boards round-trip."""
import os

import numpy as np
import torch

from skillshot_learning_amd import learner, persist


def test_models_save_names_and_round_trip(tmp_path):
    loc = str(tmp_path / "training_models")
    torch.manual_seed(0)
    a, c = learner.Actor(), learner.Critic()
    w0 = {k: v.clone() for k, v in a.state_dict().items()}
    persist.save_actor_critic_models(loc, a, c, 3)
    with torch.no_grad():
        a.l1.weight.add_(1.0)
        c.l3.bias.add_(2.0)
    persist.save_actor_critic_models(loc, a, c, 5)
    # the reference's numbering: <start>_<end>, next start = last end + 1 (:150-156)
    assert sorted(os.listdir(os.path.join(loc, "actor"))) == ["0_3_model.safetensors", "4_9_model.safetensors"]
    assert sorted(os.listdir(os.path.join(loc, "critic"))) == ["0_3_model.safetensors", "4_9_model.safetensors"]
    b, d = learner.Actor(), learner.Critic()
    assert persist.load_actor_critic_models(loc, b, d, load_index=0)
    for k, v in b.state_dict().items():
        assert torch.equal(v, w0[k]), k
    assert persist.load_actor_critic_models(loc, b, d)  # default: the latest
    assert torch.equal(b.l1.weight, a.l1.weight) and torch.equal(d.l3.bias, c.l3.bias)
    assert not persist.load_actor_critic_models(str(tmp_path / "nothing"), b, d)


def test_progress_csv_appends(tmp_path):
    loc = str(tmp_path)
    p1 = dict(epoch_ticks=[torch.tensor([10, 2000]), torch.tensor([7, 8])],
              epoch_winner=[torch.tensor([1, 0]), torch.tensor([2, 1])])
    persist.save_training_progress(loc, p1)
    persist.save_training_progress(loc, dict(epoch_ticks=[torch.tensor([5, 6])], epoch_winner=[torch.tensor([0, 2])]))
    df = persist.load_training_progress(loc)
    assert list(df.columns) == ["epoch", "game", "epoch_ticks", "epoch_winner"]
    assert df["epoch_ticks"].tolist() == [10, 2000, 7, 8, 5, 6]
    assert df["epoch_winner"].tolist() == [1, 0, 2, 1, 0, 2]
    assert df["game"].tolist() == [0, 1, 0, 1, 0, 1]


def test_boards_round_trip(tmp_path):
    rng = np.random.default_rng(0)
    seqs = [rng.integers(0, 5, size=(t, 250, 250)).astype(np.int8) for t in (3, 1, 0)]
    persist.save_training_boards(str(tmp_path), seqs)
    back = persist.load_training_boards(str(tmp_path))
    assert len(back) == 3
    for a, b in zip(seqs, back):
        assert b.dtype == np.int8 and np.array_equal(a, b)
