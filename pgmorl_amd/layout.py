"""Reference state_dict <-> flat per-task device parameter vector.

The device stores every weight TRANSPOSED ([in][out], so a lane per output unit reads
consecutive addresses) in the reference's named_parameters() order, each tensor 16-byte aligned
(offsets from pgm_param_layout, include/pgm_abi.h).  State-dict keys are the reference's
(a2c_ppo_acktr/model.py:211-254, a2c_ppo_acktr/distributions.py:78-79) for layernorm=False.
"""
import numpy as np
import torch

from ._lib import param_layout

# (state_dict key, device tensor name, transposed on device)
STATE_KEYS = [
    ('base.actor.0.weight', 'actor_w1', True),
    ('base.actor.0.bias', 'actor_b1', False),
    ('base.actor.2.weight', 'actor_w2', True),
    ('base.actor.2.bias', 'actor_b2', False),
    ('base.critic.0.weight', 'critic_w1', True),
    ('base.critic.0.bias', 'critic_b1', False),
    ('base.critic.2.weight', 'critic_w2', True),
    ('base.critic.2.bias', 'critic_b2', False),
    ('base.critic_linear.weight', 'value_w', True),
    ('base.critic_linear.bias', 'value_b', False),
    ('dist.fc_mean.weight', 'mean_w', True),
    ('dist.fc_mean.bias', 'mean_b', False),
    ('dist.logstd._bias', 'logstd', False),
]


def ref_shapes(O, A, K, H=64):
    return {
        'base.actor.0.weight': (H, O), 'base.actor.0.bias': (H,), 'base.actor.2.weight': (H, H),
        'base.actor.2.bias': (H,), 'base.critic.0.weight': (H, O), 'base.critic.0.bias': (H,),
        'base.critic.2.weight': (H, H), 'base.critic.2.bias': (H,), 'base.critic_linear.weight': (K, H),
        'base.critic_linear.bias': (K,), 'dist.fc_mean.weight': (A, H), 'dist.fc_mean.bias': (A,),
        'dist.logstd._bias': (A, 1),
    }


class ParamLayout:
    def __init__(self, O, A, K, H=64):
        self.O, self.A, self.K, self.H = O, A, K, H
        self.offsets, self.total = param_layout(O, A, K, H)
        self.shapes = ref_shapes(O, A, K, H)

    def flatten(self, tensors, dtype=np.float32):
        """Reference-shaped tensors (dict key -> array-like, e.g. a state_dict) -> flat [total] array."""
        out = np.zeros(self.total, dtype=dtype)
        for key, name, tr in STATE_KEYS:
            v = tensors[key]
            v = v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)
            if v.shape != self.shapes[key]:
                raise ValueError(f'{key}: shape {v.shape} != {self.shapes[key]}')
            if tr:
                v = v.T
            flat = np.ascontiguousarray(v, dtype=np.float64).reshape(-1)
            o = self.offsets[name]
            out[o:o + flat.size] = flat
        return out

    def unflatten(self, flat, dtype=torch.float64):
        """flat [total] -> OrderedDict of reference-shaped torch tensors (a loadable state_dict)."""
        from collections import OrderedDict
        flat = flat.detach().cpu().numpy() if isinstance(flat, torch.Tensor) else np.asarray(flat)
        sd = OrderedDict()
        for key, name, tr in STATE_KEYS:
            shp = self.shapes[key]
            n = int(np.prod(shp))
            o = self.offsets[name]
            v = flat[o:o + n].astype(np.float64)  # a fresh array: the tensor may own it
            if tr:
                v = np.ascontiguousarray(v.reshape(shp[1], shp[0]).T)
            t = torch.from_numpy(v.reshape(shp))
            sd[key] = t if t.dtype == dtype else t.to(dtype)
        return sd

    def unflatten_batch(self, flats):
        """[E, total] flat vectors -> per state_dict key (STATE_KEYS order) a C-contiguous fp64 [E, *shape] array,
        row i equal to unflatten(flats[i])[key].  A torch tensor (e.g. on the GPU) is converted and transposed
        where it lives, then copied to the host once per key."""
        if isinstance(flats, torch.Tensor):
            E = flats.shape[0]
            out = []
            for key, name, tr in STATE_KEYS:
                shp = self.shapes[key]
                n = int(np.prod(shp))
                o = self.offsets[name]
                v = flats[:, o:o + n].to(torch.float64)
                if tr:
                    v = v.reshape(E, shp[1], shp[0]).transpose(1, 2)
                out.append(v.contiguous().reshape((E,) + tuple(shp)).cpu().numpy())
            return out
        flats = np.asarray(flats)
        E = flats.shape[0]
        out = []
        for key, name, tr in STATE_KEYS:
            shp = self.shapes[key]
            n = int(np.prod(shp))
            o = self.offsets[name]
            v = flats[:, o:o + n].astype(np.float64)
            if tr:
                v = v.reshape(E, shp[1], shp[0]).transpose(0, 2, 1)
            out.append(np.ascontiguousarray(v).reshape((E,) + tuple(shp)))
        return out

    def adam_from_optimizer_state(self, opt_state):
        """torch Adam state_dict()['state'] -> (m flat, v flat, step int)."""
        if not opt_state:
            return np.zeros(self.total, np.float32), np.zeros(self.total, np.float32), 0
        ms, vs, steps = {}, {}, set()
        for i, (key, _, _) in enumerate(STATE_KEYS):
            st = opt_state.get(i)
            if st is None:  # parameter never received a gradient: torch keeps no state for it
                ms[key] = vs[key] = np.zeros(self.shapes[key])
                continue
            ms[key], vs[key] = st['exp_avg'], st['exp_avg_sq']
            steps.add(int(float(st['step'])))
        if len(steps) != 1:
            raise ValueError(f'inconsistent Adam step counts {steps}')
        return self.flatten(ms), self.flatten(vs), steps.pop()

    def adam_to_optimizer_state(self, m, v, step, dtype=torch.float64):
        ms, vs = self.unflatten(m, dtype), self.unflatten(v, dtype)
        if step == 0:
            return {}
        return {i: {'step': torch.tensor(float(step), dtype=dtype), 'exp_avg': ms[key], 'exp_avg_sq': vs[key]}
                for i, (key, _, _) in enumerate(STATE_KEYS)}
