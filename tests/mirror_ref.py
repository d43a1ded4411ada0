"""Independent pure-Python restatement of the reference's search semantics,
written directly from src/SelfPlay.jl (dict-of-nodes like the reference),
used to cross-check the C oracle's tree logic (tests only).

It shares with the oracle only the numerics contract (det_expf / Dirichlet
sampler / Philox via the oracle's exported functions, and the network
forwards); every tree rule — Q1 in-place doubling, Q2 parent-state leaf
evaluation, Q3 double softmax, Q4 root legal set, Q5 f64 pUCT, Q7 backup,
Q8 to_play bookkeeping — is re-implemented here independently.
"""
import ctypes
import math

import numpy as np

f32 = np.float32
TIE, ACTION = 2, 3


class Node:                                                     # SelfPlay.jl:62-70
    def __init__(self, prior):
        self.visit_count = 0
        self.to_play = 1
        self.prior = f32(prior)
        self.value_sum = f32(0.0)
        self.children = None
        self.hidden_state = None
        self.reward = f32(0.0)


def node_value(n):                                              # :76-82
    return f32(0.0) if n.visit_count == 0 else f32(n.value_sum / f32(n.visit_count))


class Mirror:
    def __init__(self, oracle, conf_py):
        self.o = oracle
        self.L = oracle.L
        self.c = conf_py
        self.P = len(conf_py.players)
        self.A = len(conf_py.action_space)
        self.disc = f32(conf_py.discount)

    def softmax(self, xs):
        m = xs[0]
        for x in xs[1:]:
            m = m if m > x else x
        e = [f32(self.L.ora_det_expf(float(f32(x - m)))) for x in xs]
        s = f32(0.0)
        for v in e:
            s = f32(s + v)
        return [f32(v / s) for v in e]

    def expand_node(self, node, actions, to_play, reward, policy, hidden):   # :88-96
        vals = self.softmax([policy[a - 1] for a in actions])
        node.children = {a: Node(p) for a, p in zip(actions, vals)}
        node.to_play = to_play
        node.reward = f32(reward)
        node.hidden_state = hidden

    def add_noise(self, node, gid, step):                      # :102-109
        acts = list(node.children.keys())
        noise = np.zeros(len(acts), np.float32)
        self.L.ora_dirichlet(self.o.seed, gid, step, len(acts), float(f32(self.c.dirichlet_α)),
                             noise.ctypes.data_as(ctypes.c_void_p))
        eps = f32(self.c.exploration_ϵ)
        for a, n in zip(acts, noise):
            ch = node.children[a]
            ch.prior = f32(f32(ch.prior * f32(f32(1.0) - eps)) + f32(n * eps))

    def ucb(self, parent, child, mm):                           # :171-184
        c = self.c
        pb_c = math.log2((parent.visit_count + c.pb_c_base + 1) / c.pb_c_base) + float(f32(c.pb_c_init))
        pb_c *= math.sqrt(parent.visit_count) / (child.visit_count + 1)
        prior_score = pb_c * float(child.prior)
        if child.visit_count > 0:
            q = node_value(child)
            t = f32(self.disc * q) if self.P == 1 else f32(self.disc * f32(-q))
            v = f32(child.reward + t)
            vs = f32((v - mm[0]) / f32(mm[1] - mm[0])) if mm[1] > mm[0] else v
        else:
            vs = f32(0.0)
        return f32(prior_score + float(vs))

    def select_child(self, node, mm, gid, step, sim, depth):   # :157-166
        actions = list(node.children.keys())
        scores = [self.ucb(node, node.children[a], mm) for a in actions]
        m = max(scores)
        ties = [i for i, s in enumerate(scores) if s == m]
        r = self.L.ora_rng_u32(self.o.seed, TIE, gid, step, (sim << 12) | depth)
        i = ties[(r * len(ties)) >> 32]
        return actions[i], node.children[actions[i]]

    def backpropagate(self, path, value, to_play, mm):         # :190-217
        d = self.disc
        value = f32(value)
        for node in reversed(path):
            if self.P == 1:
                node.value_sum = f32(node.value_sum + value)
            elif node.to_play == to_play:
                node.value_sum = f32(node.value_sum + value)
            else:
                node.value_sum = f32(node.value_sum - value)
            node.visit_count += 1
            u = f32(node.reward + f32(d * node_value(node)))
            mm[0] = mm[0] if mm[0] < u else u
            mm[1] = mm[1] if mm[1] > u else u
            if self.P == 1 or node.to_play != to_play:
                value = f32(node.reward + f32(d * value))
            else:
                value = f32(-node.reward)

    def run_mcts(self, obs, legal_actions, to_play, exploration, gid, step):  # :230-285
        root = Node(0.0)
        h = self.o.forward(0, obs[None, :])[0].copy()
        _, pol = self.o.forward(1, h[None, :])
        self.expand_node(root, legal_actions, to_play, 0.0, pol[0], h)
        if exploration:
            self.add_noise(root, gid, step)
        mm = [f32(np.inf), f32(-np.inf)]
        plane = self.o.plane                                     # the hidden state's board
        for it in range(self.c.num_iters):
            node, vtp, path, depth, action = root, to_play, [root], 0, 0
            while node.children is not None:
                depth += 1
                action, node = self.select_child(node, mm, gid, step, it, depth)
                path.append(node)
                vtp = ((vtp + 1 - 1) % self.P) + 1                 # mod1(vtp+1, |players|)
            parent = path[-2]
            v, pl = self.o.forward(1, parent.hidden_state[None, :])
            parent.hidden_state *= f32(2.0)                         # Q1: in place
            sa = np.concatenate([parent.hidden_state, np.full(plane, f32(action / self.A), np.float32)])
            nh, r = self.o.forward(2, sa[None, :])
            self.expand_node(node, legal_actions, vtp, r[0, 0], pl[0], nh[0].copy())
            self.backpropagate(path, v[0, 0], vtp, mm)
        return root

    def select_action(self, root, temperature, gid, step):     # :293-306 (T = 1 / 0 rules)
        acts = list(root.children.keys())
        cnt = [root.children[a].visit_count for a in acts]
        r = self.L.ora_rng_u32(self.o.seed, ACTION, gid, step, 0)
        if temperature == 0.0:
            return acts[int(np.argmax(cnt))]
        tot = sum(cnt)
        t = (r * tot) >> 32
        cum = 0
        for a, n in zip(acts, cnt):
            cum += n
            if cum > t:
                return a
        return acts[-1]

    def search(self, obs, legal, to_play, exploration, game_offset, step, temperature=1.0):
        G = obs.shape[0]
        cv = np.zeros((G, self.A), np.float32)
        rv = np.zeros(G, np.float32)
        act = np.zeros(G, np.int32)
        roots = []
        for g in range(G):
            la = [a + 1 for a in np.flatnonzero(legal[g])]
            root = self.run_mcts(obs[g], la, int(to_play[g]), exploration, game_offset + g, step)
            tot = sum(ch.visit_count for ch in root.children.values())
            for a, ch in root.children.items():
                cv[g, a - 1] = f32(ch.visit_count / tot)
            rv[g] = node_value(root)
            act[g] = self.select_action(root, temperature, game_offset + g, step)
            roots.append(root)
        return cv, rv, act, roots
