"""NeuralNet plug-in for Splendor (NNet.py:1-9 + GenericNNetWrapper.predict/checkpoints).

Inference only: training (GenericNNetWrapper.train, losses, optimiser) is outside the
self-play hot path. Checkpoints are read with torch.load(weights_only=True);
files that pickle whole model objects (like the reference's genbu.pt) are refused by that
loader and are reported, never unpickled.
"""
import os

import numpy as np
import torch

from .nnet import SplendorNNet, remap_policy_head


class NNetWrapper:
    def __init__(self, game, nn_args=None, use_exchange=True, device=None, seed=0):
        self.args = nn_args or {}
        self.device = torch.device(device) if device else game.engine.device
        torch.manual_seed(seed)
        self.nnet = SplendorNNet(game.num_players).to(self.device).eval()
        self.action_size = game.getActionSize()
        self.rows = game.getBoardSize()[0]

    @torch.no_grad()
    def predict(self, board, valid_actions):
        """GenericNNetWrapper.predict (:141-168): (exp(log_pi)[409], tanh(v)[n]) as numpy."""
        b = torch.as_tensor(np.asarray(board, dtype=np.float32), device=self.device).reshape(1, self.rows, 7)
        va = torch.as_tensor(np.asarray(valid_actions, dtype=bool), device=self.device).reshape(1, -1)
        log_pi, v, _ = self.nnet(b, va)
        return torch.exp(log_pi)[0].cpu().numpy(), v[0].cpu().numpy()

    def save_checkpoint(self, folder="checkpoint", filename="checkpoint.pt", additional_keys=None):
        os.makedirs(folder, exist_ok=True)
        data = {"state_dict": self.nnet.state_dict()}
        data.update(additional_keys or {})
        torch.save(data, os.path.join(folder, filename))

    def load_checkpoint(self, folder="checkpoint", filename="checkpoint.pt"):
        path = os.path.join(folder, filename)
        try:
            data = torch.load(path, map_location=self.device, weights_only=True)
        except Exception as e:  # refused by the safe loader: never fall back to unpickling
            raise RuntimeError(f"{path}: not loadable with torch.load(weights_only=True) ({type(e).__name__})") from e
        sd = data["state_dict"] if isinstance(data, dict) and "state_dict" in data else data
        self.nnet.load_state_dict(remap_policy_head(sd))   # 406-action checkpoints -> 409
        self.nnet.eval()
        return data
