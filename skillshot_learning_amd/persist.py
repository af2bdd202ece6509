"""On-disk formats of the learner (SkillshotLearner.py:123-204).

Same directory layout and names as the reference, under `save_location`
(default "training_models"):

    actor/<start>_<end>_model.safetensors     (reference: .h5 Keras models)
    critic/<start>_<end>_model.safetensors
    training_progress/training_progress.csv   (pandas, append mode)
    training_boards/training_boards.npz       (reference: training_boards.npy)

Deliberate differences, each because the reference's own path cannot run as
written or needs a library absent here:
* models are torch state dicts in safetensors (h5py / Keras are not
  installed); the epoch-range file naming and "continue from the last end"
  numbering are the reference's (:139-160);
* the reference sorts file names with `int(x.split("_"[1]))` (:129, :150),
  which raises IndexError as soon as a directory holds a file; the evident
  intent — order by the leading epoch number — is what is implemented;
* the progress CSV holds one row per (epoch, game) with the episode's ticks
  and winner (the batched engine plays N games per epoch); the reference
  builds its DataFrame from three lists of which `epoch_board_sequences` is
  empty unless boards are saved, which makes pandas raise for any saved epoch;
* boards go to an .npz with one int8 [ticks, 250, 250] array per epoch (the
  reference's ragged list needs a pickled object array; values are 0-4).
"""
import os

import numpy as np
import torch

ACTOR_DIR, CRITIC_DIR = "actor", "critic"
PROGRESS_DIR, BOARDS_DIR = "training_progress", "training_boards"


def _epoch_sorted(files):
    return sorted(files, key=lambda x: int(x.split("_")[0]))


def save_actor_critic_models(save_location, actor, critic, epochs):
    """save_actor_critic_models (:139-160): one file per net named
    <start>_<end>_model, start continuing from the last saved end + 1."""
    from safetensors.torch import save_file
    paths = []
    for model, dir_name in ((actor, ACTOR_DIR), (critic, CRITIC_DIR)):
        loc = os.path.join(save_location, dir_name)
        os.makedirs(loc, exist_ok=True)
        files = _epoch_sorted([f for f in os.listdir(loc) if f.endswith("_model.safetensors")])
        start = 0 if not files else int(files[-1].split("_")[1]) + 1
        name = f"{start}_{start + int(epochs)}_model.safetensors"
        state = {k: v.detach().to("cpu").contiguous() for k, v in model.state_dict().items()}
        save_file(state, os.path.join(loc, name))
        paths.append(os.path.join(loc, name))
    print("Actor and Critic Saved.")
    return paths


def load_actor_critic_models(save_location, actor, critic, load_index=-1):
    """load_actor_critic_models (:123-137): the load_index-th file (epoch
    order) of each net; False (after printing the location) if a net has none."""
    from safetensors.torch import load_file
    for model, dir_name in ((actor, ACTOR_DIR), (critic, CRITIC_DIR)):
        loc = os.path.join(save_location, dir_name)
        files = _epoch_sorted([f for f in os.listdir(loc) if f.endswith("_model.safetensors")]) \
            if os.path.isdir(loc) else []
        if not files:
            print("Failed to load: ", loc)
            return False
        state = load_file(os.path.join(loc, files[load_index]))
        dev = next(model.parameters()).device
        with torch.no_grad():
            model.load_state_dict({k: v.to(dev) for k, v in state.items()})
    return True


def progress_frame(total_progress):
    """One row per (epoch, game): epoch, game, epoch_ticks, epoch_winner."""
    import pandas as pd
    rows = []
    for e, (t, w) in enumerate(zip(total_progress["epoch_ticks"], total_progress["epoch_winner"])):
        t = np.atleast_1d(np.asarray(torch.as_tensor(t).cpu()))
        w = np.atleast_1d(np.asarray(torch.as_tensor(w).cpu()))
        for gi in range(t.shape[0]):
            rows.append((e, gi, int(t[gi]), int(w[gi])))
    return pd.DataFrame(rows, columns=["epoch", "game", "epoch_ticks", "epoch_winner"])


def save_training_progress(save_location, total_progress):
    """save_training_progress (:162-172): pandas to_csv in append mode."""
    loc = os.path.join(save_location, PROGRESS_DIR)
    os.makedirs(loc, exist_ok=True)
    path = os.path.join(loc, "training_progress.csv")
    progress_frame(total_progress).to_csv(path, mode="a")
    print("Training Progress Saved")
    return path


def load_training_progress(save_location):
    """load_training_progress (:174-179): the CSV as a DataFrame (each append
    repeats the header row, as pandas' append mode writes it; those rows are
    dropped)."""
    import pandas as pd
    df = pd.read_csv(os.path.join(save_location, PROGRESS_DIR, "training_progress.csv"), index_col=0)
    df = df[df["epoch"] != "epoch"]
    return df.astype({"epoch": int, "game": int, "epoch_ticks": int, "epoch_winner": int}).reset_index(drop=True)


def save_training_boards(save_location, epoch_board_list):
    """save_training_boards (:181-192): every epoch's board sequence, one file
    (overwritten, as the reference's np.save is)."""
    loc = os.path.join(save_location, BOARDS_DIR)
    os.makedirs(loc, exist_ok=True)
    path = os.path.join(loc, "training_boards.npz")
    np.savez_compressed(path, **{f"epoch_{k}": np.asarray(b, dtype=np.int8) for k, b in enumerate(epoch_board_list)})
    print("Training Boards Saved")
    return path


def load_training_boards(save_location):
    """load_training_boards (:194-204): the list of per-epoch [ticks, 250, 250] boards."""
    d = np.load(os.path.join(save_location, BOARDS_DIR, "training_boards.npz"))
    return [d[f"epoch_{k}"] for k in range(len(d.files))]
