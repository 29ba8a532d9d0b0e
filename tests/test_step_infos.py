"""SalpVecEnv's lazy infos (vec_env.StepInfos) on the CPU: the dicts SB3 and
the reference's TensorboardCallback (src/tensorboard_callback.py:72-123) read,
built from one step's host arrays only when accessed."""
import numpy as np

from grasp_lab_salp_amd._abi import EPISODE_METRIC_KEYS, INFO, REWARD_COMPONENT_KEYS
from grasp_lab_salp_amd.vec_env import StepInfos, _EmptyInfos


def _infos():
    n, od = 6, 10
    info = np.arange(n * len(INFO), dtype=np.float64).reshape(n, len(INFO))
    tobs = np.arange(n * od, dtype=np.float32).reshape(n, od)
    term = np.array([0, 1, 0, 0, 1, 0], bool)
    trunc = np.array([0, 0, 1, 0, 1, 0], bool)
    return StepInfos(info, tobs, term, trunc, term | trunc, 1.5), info, tobs


def test_not_done_env_has_reward_components_only():
    infos, info, _ = _infos()
    d = infos[0]
    assert list(d) == list(REWARD_COMPONENT_KEYS)
    assert d["rewards/track"] == info[0, INFO["rewards/track"]]
    assert "episode" not in d and "terminal_observation" not in d


def test_done_env_has_monitor_and_timelimit_entries():
    infos, info, tobs = _infos()
    d1, d2, d4 = infos[1], infos[2], infos[4]
    assert d1["TimeLimit.truncated"] is False          # terminated
    assert d2["TimeLimit.truncated"] is True           # truncated only
    assert d4["TimeLimit.truncated"] is False          # both: SB3 counts it as terminated
    assert np.array_equal(d2["terminal_observation"], tobs[2])
    assert d2["episode"] == {"r": round(info[2, INFO["ep_return"]], 6), "l": int(info[2, INFO["ep_len"]]), "t": 1.5}
    assert all(k in d2 for k in EPISODE_METRIC_KEYS)
    assert list(infos.done_indices) == [1, 2, 4]


def test_sequence_protocol_and_cached_edits():
    infos, _, _ = _infos()
    assert len(infos) == 6 and len(list(infos)) == 6
    assert infos[-1] is infos[5]
    infos[3]["custom"] = 7          # a consumer's edit sticks (SB3 wrappers add keys)
    assert infos[3]["custom"] == 7
    assert [d["rewards/track"] for d in infos[1:3]] == [infos[1]["rewards/track"], infos[2]["rewards/track"]]
    scan = [i for i, d in enumerate(infos) if "episode" in d]     # the reference callback's scan
    assert scan == [1, 2, 4]


def test_detach_keeps_values_after_the_buffer_changes():
    infos, info, tobs = _infos()
    infos._detach()
    info[:] = -1
    tobs[:] = -1
    assert infos[2]["rewards/track"] == 2 * len(INFO) + INFO["rewards/track"]
    assert infos[2]["terminal_observation"][0] == 20


def test_empty_infos():
    e = _EmptyInfos(None, None, np.zeros(3, bool), np.zeros(3, bool), np.zeros(3, bool), 0.0)
    assert list(e) == [{}, {}, {}]
