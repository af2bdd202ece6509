"""numpy (fp64) restatement of the reference learner's arithmetic: the Keras
nets, losses, gradients and optimiser of SkillshotLearner.py.

TEST INFRASTRUCTURE ONLY (see oracle/oracle.py): the checker for the fp32 and
bf16 learner kernels and the torch path, never the product.

The algorithm lives in TensorFlow 2.x Keras, which the reference imports
(`SkillshotLearner.py:5-11`) without pinning a version and which is absent
here; what follows restates Keras' published semantics at the reference's
call sites, so parity is anchored on those call sites (no golden vectors for
the nets exist anywhere in the reference):

  * Dense(units, activation): y = act(x @ kernel + bias), kernel [in, out]
    (here stored torch-style as W [out, in], y = x W^T + b).
      actor  Dense(256, relu) -> Dense(128, relu) -> Dense(2, tanh)      (:79-89)
      critic Dense(256, relu) -> Dropout(0.2) -> concatenate([h, action])
             -> Dense(128, relu) -> Dense(1, linear)                      (:104-114)
  * Dropout(rate=0.2) in training: inverted dropout, kept units x 1/(1-rate)
    (keras.layers.Dropout); inactive at inference (the actor step calls
    the critic without training=True, :397).
  * critic.compile(optimizer="adam", loss="mse") (:118) + fit(batch_size=16)
    (:434): loss = mean over the batch of (q - y)^2 (one output unit), so
    dL/dq = 2 (q - y) / B.
  * model_actor_fit_step (:386-417): tape.gradient(action, actor weights,
    output_gradients = -dQ/da) = the gradient of -sum_b Q(s_b, mu(s_b))
    with the critic fixed.
  * Adam (tf.keras.optimizers.Adam(), :68): m += (g - m)(1 - b1),
    v += (g^2 - v)(1 - b2), alpha = lr sqrt(1 - b2^t) / (1 - b1^t),
    w -= m alpha / (sqrt(v) + eps); lr 1e-3, b1 0.9, b2 0.999, eps 1e-7.

Parameters are dicts of fp64 arrays with torch's names and shapes
(l1.weight [256, 12], l1.bias, l2.weight [128, 256 or 258], l2.bias,
l3.weight [n_out, 128], l3.bias); gradients use the same keys.
"""
import numpy as np

NAMES = ("l1.weight", "l1.bias", "l2.weight", "l2.bias", "l3.weight", "l3.bias")
DROP_SCALE = 1.0 / (1.0 - 0.2)


def from_module(module):
    """fp64 numpy copies of a torch module's parameters"""
    return {k: v.detach().double().cpu().numpy() for k, v in module.state_dict().items()}


def relu(x):
    return np.maximum(x, 0.0)


def actor_forward(P, s):
    """model_define_actor (:70-96): s [B, 12] -> (action [B, 2], cache)"""
    z1 = s @ P["l1.weight"].T + P["l1.bias"]
    h1 = relu(z1)
    z2 = h1 @ P["l2.weight"].T + P["l2.bias"]
    h2 = relu(z2)
    a = np.tanh(h2 @ P["l3.weight"].T + P["l3.bias"])
    return a, dict(s=s, h1=h1, h2=h2, a=a)


def critic_forward(P, s, a, keep=None):
    """model_define_critic (:98-121): (s, a) -> (q [B], cache); keep = Dropout
    keep-mask [B, 256] in training, None at inference"""
    h1 = relu(s @ P["l1.weight"].T + P["l1.bias"])
    hd = h1 * keep * DROP_SCALE if keep is not None else h1
    x2 = np.concatenate([hd, a], axis=1)
    h2 = relu(x2 @ P["l2.weight"].T + P["l2.bias"])
    q = (h2 @ P["l3.weight"].T + P["l3.bias"])[:, 0]
    return q, dict(s=s, a=a, h1=h1, hd=hd, x2=x2, h2=h2, keep=keep)


def critic_backward(P, c, dq):
    """gradients of sum_b dq_b q_b w.r.t. the critic's parameters, and dq/da"""
    g = {}
    g["l3.weight"] = dq[None, :] @ c["h2"]
    g["l3.bias"] = np.array([dq.sum()])
    dz2 = (dq[:, None] * P["l3.weight"]) * (c["h2"] > 0)
    g["l2.weight"] = dz2.T @ c["x2"]
    g["l2.bias"] = dz2.sum(0)
    dx2 = dz2 @ P["l2.weight"]
    dhd, da = dx2[:, :256], dx2[:, 256:]
    dh1 = dhd * c["keep"] * DROP_SCALE if c["keep"] is not None else dhd
    dz1 = dh1 * (c["h1"] > 0)
    g["l1.weight"] = dz1.T @ c["s"]
    g["l1.bias"] = dz1.sum(0)
    return g, da


def critic_grads(P, s, a, y, keep, global_batch=None):
    """critic.fit step (:434): MSE loss mean over the (global) batch; returns
    (grads, loss)"""
    B = s.shape[0] if global_batch is None else global_batch
    q, c = critic_forward(P, s, a, keep)
    g, _ = critic_backward(P, c, 2.0 * (q - y) / B)
    return g, float(((q - y) ** 2).sum() / B)


def actor_grads(A, C, s):
    """model_actor_fit_step (:386-417): gradient of -sum_b Q(s_b, mu(s_b)),
    critic at inference; returns (grads, sum_b Q)"""
    act, ca = actor_forward(A, s)
    q, cc = critic_forward(C, s, act, None)
    _, dqda = critic_backward(C, cc, np.ones_like(q))
    dz3 = -dqda * (1.0 - act * act)
    g = {}
    g["l3.weight"] = dz3.T @ ca["h2"]
    g["l3.bias"] = dz3.sum(0)
    dz2 = (dz3 @ A["l3.weight"]) * (ca["h2"] > 0)
    g["l2.weight"] = dz2.T @ ca["h1"]
    g["l2.bias"] = dz2.sum(0)
    dz1 = (dz2 @ A["l2.weight"]) * (ca["h1"] > 0)
    g["l1.weight"] = dz1.T @ s
    g["l1.bias"] = dz1.sum(0)
    return g, float(q.sum())


def target_y(TA, TC, s2, r, d, gamma):
    """north_star extension (no reference row): y = r + gamma (1 - d) Q'(s', mu'(s'))"""
    a2, _ = actor_forward(TA, s2)
    q2, _ = critic_forward(TC, s2, a2, None)
    return r + gamma * (1.0 - d) * q2


class Adam:
    """tf.keras.optimizers.Adam() (:68) on a parameter dict"""

    def __init__(self, P, lr=1e-3, b1=0.9, b2=0.999, eps=1e-7):
        self.lr, self.b1, self.b2, self.eps = lr, b1, b2, eps
        self.m = {k: np.zeros_like(v) for k, v in P.items()}
        self.v = {k: np.zeros_like(v) for k, v in P.items()}
        self.t = 0

    def step(self, P, g):
        self.t += 1
        alpha = self.lr * np.sqrt(1.0 - self.b2 ** self.t) / (1.0 - self.b1 ** self.t)
        for k in P:
            self.m[k] += (g[k] - self.m[k]) * (1.0 - self.b1)
            self.v[k] += (g[k] * g[k] - self.v[k]) * (1.0 - self.b2)
            P[k] = P[k] - self.m[k] * alpha / (np.sqrt(self.v[k]) + self.eps)
        return P


def soft_update(T, P, tau):
    """north_star extension: target += tau (online - target)"""
    for k in T:
        T[k] = T[k] + tau * (P[k] - T[k])
    return T
