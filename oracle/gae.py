"""CPU restatement of SB3's GAE / return computation (test infrastructure only).

TEST INFRASTRUCTURE ONLY — imported by tests/ and never by the product
package.  The reference trains with sb3-contrib's RecurrentPPO
(src/train_robot_recurrent_ppo.py:85-107, gamma 0.99, gae_lambda 0.95 at
:94-95), whose rollout buffer inherits
``stable_baselines3.common.buffers.RolloutBuffer.compute_returns_and_advantage``
(stable-baselines3 >= 2.0 per requirements.txt:6-7; the version is not pinned
and the package is not installed here, so this restatement of its published
algorithm is "parity unpinned": no reference test or fixture covers it).
``collect_rollouts``'s timeout bootstrap (``rewards[idx] += gamma *
terminal_value`` for truncated episodes) is restated in :func:`bootstrap_timeouts`.

Arrays are float32 ``[n_steps, n_envs]`` as in SB3; the arithmetic below is the
SB3 expression evaluated by NumPy 2, so Python-float coefficients become
float32 (NEP 50).
"""
import numpy as np


def compute_returns_and_advantage(rewards, values, episode_starts, last_values, dones,
                                  gamma=0.99, gae_lambda=0.95):
    """Returns (advantages, returns), float32 [n_steps, n_envs]."""
    rewards = np.asarray(rewards, np.float32)
    values = np.asarray(values, np.float32)
    episode_starts = np.asarray(episode_starts, np.float32)
    last_values = np.asarray(last_values, np.float32).flatten()
    dones = np.asarray(dones)
    n_steps = rewards.shape[0]
    advantages = np.zeros_like(rewards)
    last_gae_lam = 0
    for step in reversed(range(n_steps)):
        if step == n_steps - 1:
            next_non_terminal = 1.0 - dones.astype(np.float32)
            next_values = last_values
        else:
            next_non_terminal = 1.0 - episode_starts[step + 1]
            next_values = values[step + 1]
        delta = rewards[step] + gamma * next_values * next_non_terminal - values[step]
        last_gae_lam = delta + gamma * gae_lambda * next_non_terminal * last_gae_lam
        advantages[step] = last_gae_lam
    returns = advantages + values
    return advantages, returns


def bootstrap_timeouts(rewards, truncated, terminated, terminal_values, gamma=0.99):
    """SB3 OnPolicyAlgorithm.collect_rollouts: for envs whose episode ended by
    truncation (``TimeLimit.truncated`` = truncated and not terminated), add
    gamma * V(terminal observation) to that step's reward.  float32."""
    r = np.asarray(rewards, np.float32).copy()
    mask = np.asarray(truncated, bool) & ~np.asarray(terminated, bool)
    tv = np.asarray(terminal_values, np.float32)
    r[mask] = r[mask] + np.float32(gamma) * tv[mask]
    return r
