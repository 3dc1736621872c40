"""Schedule-probability normalisation (reference: ``common/common_functionalities.py:12-55``)."""
import numpy as np

ACCURACY = float(np.sqrt(np.finfo(np.float64).eps))


def normalize_scheduling_probabilities(input_list) -> list:
    """Return probabilities summing to one: all-zero -> uniform (rounded to 1e-10), otherwise divide by the
    sum (rounded) unless already within ``ACCURACY``; the residual goes to the first element that can absorb it."""
    probs = list(input_list)
    if len(probs) == 0:
        return []
    total = sum(probs)
    if total == 0:
        out = [round(1 / len(probs), 10)] * len(probs)
    elif abs(1 - total) > ACCURACY:
        out = [round(p / total, 10) for p in probs]
    else:
        out = probs.copy()
    residual = 1 - sum(out)
    if residual != 0:
        i = 0
        while out[i] + residual < 0:
            i += 1
        out[i] = out[i] + residual
    assert abs(1 - sum(out)) < ACCURACY, "sum of probabilities != 1"
    return out


REFERENCE_SCHEDULE_THRESHOLD = 0.1  # src/rlsp/agents/simple_ddpg.py:130


def schedule_threshold(cfg: dict, n_pad: int) -> float:
    """Post-processing threshold of the schedule rows.  Default: the reference's fixed 0.1
    (``simple_ddpg.py:130``).  Opt-in agent key ``schedule_threshold`` (new; docs/DEVIATIONS.md): a float, or
    ``auto`` = 0.1 * 24 / n_pad -- the reference's value at its 24-node padding, scaled with 1/n so that a row of
    ~n comparable weights (each ~1/n after normalising) is not zeroed wholesale at 50-200 nodes, which turns every
    row into the uniform schedule and leaves the critic no action variation (profiles/learning_curves.md)."""
    v = cfg.get("schedule_threshold", None)
    if v is None:
        return REFERENCE_SCHEDULE_THRESHOLD
    if isinstance(v, str):
        if v.strip().lower() == "auto":
            return REFERENCE_SCHEDULE_THRESHOLD if n_pad <= 24 else 2.4 / float(n_pad)
        v = float(v)
    v = float(v)
    if not 0.0 <= v < 1.0:
        raise ValueError(f"schedule_threshold must be in [0, 1) or 'auto', got {v}")
    return v


def threshold_normalize(action: np.ndarray, slice_len: int, threshold: float = 0.1, passes: int = 2) -> np.ndarray:
    """Per slice of ``slice_len``: zero entries below ``threshold`` then normalise; repeated ``passes`` times.

    ``passes=2`` is SimpleDDPG.post_process_actions (simple_ddpg.py:374-395); ``passes=1`` is
    ActionScheduleProcessor (action_norm_processor.py:18-42)."""
    action = np.asarray(action, dtype=np.float64)
    assert action.shape[0] % slice_len == 0
    out = np.empty_like(action)
    for s in range(action.shape[0] // slice_len):
        probs = action[s * slice_len:(s + 1) * slice_len]
        for _ in range(passes):
            probs = np.array(normalize_scheduling_probabilities([p if p >= threshold else 0 for p in probs]))
        out[s * slice_len:(s + 1) * slice_len] = probs
    return out


class ActionScheduleProcessor:
    """Single-pass threshold + normalise (reference ``src/rlsp/envs/action_norm_processor.py``)."""

    def __init__(self, num_nodes, num_sfcs, num_sfs, schedule_threshold=0.1):
        self.num_nodes = num_nodes
        self.num_sfcs = num_sfcs
        self.num_sfs = num_sfs
        self.schedule_threshold = schedule_threshold

    def process_action(self, action):
        assert len(action) == self.num_nodes * self.num_sfcs * self.num_sfs * self.num_nodes, "wrong dimensions"
        return threshold_normalize(action, self.num_nodes, self.schedule_threshold, passes=1)
