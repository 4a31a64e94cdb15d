"""Parametric (continuous) estimators on MI355X: LinearRegression,
LogisticRegression, NeuralNetwork.

Each class mirrors its reference counterpart (same name, constructor, config
keys, ``fit`` / ``get_prob`` / ``sample`` / ``save_model`` / ``load_model``
semantics and errors):

* ``LinearRegression``   -- cbn/parameter_learning/linear_regression.py:11-134
* ``LogisticRegression`` -- cbn/parameter_learning/logistIc_regression.py:11-141
* ``NeuralNetwork``      -- cbn/parameter_learning/neural_network.py:21-165

Training (``_fit``) is the reference's own loop -- torch autograd + the
configured torch optimizer over the same modules -- since parameter learning
is not the accelerated path.  Density evaluation (``get_prob``) and the
factors these models contribute to ``BayesianNetwork.infer`` run in the HIP
kernels of ``csrc/cbn_param.hip`` (``cbn_param_eval``,
``cbn_plan_create_param``): the model is packed once per fit/load into a flat
fp32 device buffer ``[W_0, b_0, W_1, b_1, ...]`` (nn.Linear layout, W
row-major [out][in]).  ``scale`` (= exp(log_sigma) / exp(log_scale)) and the
Gaussian normaliser are computed on the host in float32 with torch CPU ops,
in the reference's order (linear_regression.py:87-95).
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Tuple

import torch
from torch import nn
from tqdm import tqdm

from .. import _native
from ..base.parameter_learning import BaseParameterLearningEstimator, bump_generation


def config_torch_optimizer(model, config: Dict = None):
    """cbn/parameter_learning/utils.py:6-13 (``config=None`` raises AttributeError, as there)."""
    optimizer_name = config.get("name", "Adam")
    optimizer_params = config.get("params", {})
    optimizer_class = getattr(torch.optim, optimizer_name)
    return optimizer_class(model.parameters(), **optimizer_params)


activation_map = {
    "relu": nn.ReLU,
    "tanh": nn.Tanh,
    "sigmoid": nn.Sigmoid,
    "leakyrelu": nn.LeakyReLU,
    "gelu": nn.GELU,
    "elu": nn.ELU,
}
_ACT_ID = {nn.Tanh: "tanh", nn.ReLU: "relu", nn.Sigmoid: "sigmoid", nn.LeakyReLU: "leakyrelu", nn.GELU: "gelu",
           nn.ELU: "elu"}


class _Parametric(BaseParameterLearningEstimator):
    """Shared device side of the three estimators: the packed model and the
    ``cbn_param_eval`` / ``cbn_plan_create_param`` descriptors."""

    family = _native.CBN_FAMILY_LOGISTIC
    bias_only_root = False  # LinearRegression: query=None -> mu = bias

    def __init__(self, config: Dict, **kwargs):
        super().__init__(config, **kwargs)
        self._packed: Optional[Tuple[torch.Tensor, list, int, float, float]] = None

    # ---- model description (subclasses) ----
    def _linears(self) -> List[nn.Linear]:
        raise NotImplementedError

    def _activation_name(self) -> Optional[str]:
        return None

    def _log_scale(self) -> torch.Tensor:
        raise NotImplementedError

    # ---- packing ----
    def _invalidate(self):
        self._packed = None
        bump_generation(self)  # cached inference plans hold the old packed weights

    def _scale_norm(self) -> Tuple[float, float]:
        """sigma / s and the Gaussian normaliser as the reference computes them
        in float32 (linear_regression.py:87-95; logistIc_regression.py:90-98)."""
        ls = self._log_scale().detach().to("cpu", torch.float32)
        scale = torch.exp(ls)
        if self.family == _native.CBN_FAMILY_GAUSS:
            norm = 1 / (scale * torch.sqrt(torch.tensor(2 * torch.pi)))
            return float(scale), float(norm)
        return float(scale), 0.0

    def packed(self, device=None):
        """(weights [flat fp32 device], widths, act id, scale, norm), built once per fit/load."""
        if self._packed is None or (device is not None and self._packed[0].device != torch.device(device)):
            lins = self._linears()
            if not lins:
                raise RuntimeError("Model not initialized. Train or initialize the model before loading.")
            dev = torch.device(device) if device is not None else lins[0].weight.device
            parts, widths = [], [lins[0].in_features]
            for lin in lins:
                parts += [lin.weight.detach().reshape(-1), lin.bias.detach().reshape(-1)]
                widths.append(lin.out_features)
            w = torch.cat([p.to(torch.float32) for p in parts]).to(dev).contiguous()
            act = _native.CBN_ACT.get(self._activation_name() or "", 0) if len(lins) > 1 else 0
            scale, norm = self._scale_norm()
            self._packed = (w, widths, act, scale, norm)
        return self._packed

    def model_desc(self, root: bool = False, device=None) -> Tuple[_native.ParamModel, torch.Tensor]:
        """``cbn_param_model`` of this estimator as ``get_prob`` evaluates it.

        ``root``: the model of the query-free call (node.py:197-198):
        LinearRegression's mu is its bias (linear_regression.py:84-89), given
        here as the linear model [0, b] on the constant input 1; the logistic
        models run on the constant input 1 (neural_network.py:111-114)."""
        w, widths, act, scale, norm = self.packed(device)
        if len(widths) - 1 > _native.CBN_MAX_MODEL_LAYERS or max(widths) > _native.CBN_MAX_MODEL_WIDTH:
            raise _native.NativeError(
                f"model shape {widths} beyond the kernel limits ({_native.CBN_MAX_MODEL_LAYERS} layers, "
                f"{_native.CBN_MAX_MODEL_WIDTH} units per layer)")
        if root and self.bias_only_root:
            w = torch.stack([torch.zeros((), dtype=torch.float32, device=w.device), w[widths[0]]]).contiguous()
            widths = [1, 1]
        m = _native.ParamModel()
        m.family = self.family
        m.n_layers = len(widths) - 1
        if m.n_layers <= _native.CBN_MAX_LAYERS:
            for i, v in enumerate(widths):
                m.width[i] = v
        else:  # deeper models: the widths array (kept alive with the struct)
            arr = (ctypes.c_int32 * len(widths))(*widths)
            m.widths = ctypes.cast(arr, ctypes.POINTER(ctypes.c_int32))
            m._widths_keep = arr
        m.act = act
        m.weights = w.data_ptr()
        m.scale = scale
        m.norm = norm
        return m, w

    # ---- evaluation ----
    def _get_prob(self, point_to_evaluate: torch.Tensor, query: torch.Tensor = None):
        """pdf [n_queries, n_points] of the node at ``point_to_evaluate`` given
        mu = model(query.squeeze(-1)) (or the query-free mean)."""
        dev = _native.require_gpu(self.device)
        m, w = self.model_desc(device=dev)
        pts = point_to_evaluate.to(device=dev, dtype=torch.float32)
        q = None
        if query is not None:
            q = query.squeeze(-1).to(device=dev, dtype=torch.float32)
            if q.dim() == 1:
                q = q.unsqueeze(-1) if m.width[0] == 1 else q.unsqueeze(0)
            if q.dim() != 2 or q.shape[1] != m.width[0]:
                raise RuntimeError(f"mat1 and mat2 shapes cannot be multiplied ({tuple(q.shape)} and "
                                   f"{m.width[0]}x{m.width[1]})")
            n = max(q.shape[0], pts.shape[0])
            if q.shape[0] != n:
                q = q.expand(n, -1)
            q = q.contiguous()
        else:
            n = pts.shape[0]
        if pts.dim() == 1:
            pts = pts.unsqueeze(0)
        if pts.shape[0] != n:
            pts = pts.expand(n, -1)
        pts = pts.contiguous()
        out = torch.empty((n, pts.shape[1]), dtype=torch.float32, device=dev)
        with torch.cuda.device(dev):
            _native.check(_native.load().cbn_param_eval(
                ctypes.byref(m), _native.ptr(pts), n, pts.shape[1], _native.ptr(q) if q is not None else None,
                1 if (query is None and self.bias_only_root) else 0, _native.ptr(out), _native.stream_ptr(dev)),
                "cbn_param_eval")
        return out

    def eval_grid(self, parents_query: torch.Tensor, domains: torch.Tensor) -> torch.Tensor:
        """pdf[i, c, v] = pdf(domains[i, v]; mu(parents_query[i, :, c])) for all i, c at once
        (the per-query loop of node.py:177-186 as one kernel call)."""
        n, k, combos = parents_query.shape
        nv = domains.shape[1]
        q = parents_query.permute(0, 2, 1).reshape(n * combos, k, 1)
        pts = domains[:n].unsqueeze(1).expand(n, combos, nv).reshape(n * combos, nv)
        return self._get_prob(pts, q).view(n, combos, nv)


class LinearRegression(_Parametric):
    """linear_regression.py:11-134: Gaussian N(x; W q + b, exp(log_sigma))."""

    family = _native.CBN_FAMILY_GAUSS
    bias_only_root = True

    def __init__(self, config: Dict, **kwargs):
        super().__init__(config, **kwargs)
        self._setup_model(config, **kwargs)
        self.linear_model = None
        self.log_sigma = None

    def _setup_model(self, config: Dict, **kwargs):
        self.config_optimizer = config.get("optimizer")
        self.n_epochs = config.get("train", {}).get("n_epochs", 1000)

    def _linears(self):
        return [self.linear_model] if self.linear_model is not None else []

    def _log_scale(self):
        return self.log_sigma

    def _fit(self, node_data: torch.Tensor, parents_data: torch.Tensor = None):
        """linear_regression.py:25-76 (the root model regresses the node on itself)."""
        device = self.device
        if parents_data is not None:
            input_dim = parents_data.shape[0]
            queries = parents_data.transpose(0, 1).to(device).to(torch.float32)
        else:
            input_dim = 1
            queries = node_data.unsqueeze(1).to(device).to(torch.float32)
        if self.linear_model is None:
            self.linear_model = nn.Linear(input_dim, 1).to(device).to(torch.float32)
            self.log_sigma = nn.Parameter(torch.log(torch.tensor(1.0, device=device)))
        targets = node_data.to(device).unsqueeze(1)
        optimizer = config_torch_optimizer(self.linear_model, self.config_optimizer)
        bar = tqdm(range(self.n_epochs), desc="training linear regression...") if self.if_log else range(self.n_epochs)
        for _ in bar:
            optimizer.zero_grad()
            mu = self.linear_model(queries)
            sigma = torch.exp(self.log_sigma)
            loss = (0.5 * torch.log(torch.tensor(2 * torch.pi, device=device)) + self.log_sigma
                    + 0.5 * ((targets - mu) / sigma) ** 2).mean()
            loss.backward()
            optimizer.step()
            if self.if_log:
                bar.set_postfix(loss=f"{loss.item():.4f}")
        self._invalidate()

    def _sample(self, N: int, **kwargs) -> torch.Tensor:
        """linear_regression.py:98-115."""
        query = kwargs.get("query")
        sigma = torch.exp(self.log_sigma)
        if query is not None:
            mu = self.linear_model(query.squeeze(-1).to(self.device))
            return torch.normal(mu.expand(mu.shape[0], N), sigma).detach()
        mu = self.linear_model.weight.new_zeros((1,)) + self.linear_model.bias.to(self.device)
        return torch.normal(mu.expand(N), sigma).detach()

    def save_model(self, path: str):
        torch.save({"linear_state_dict": self.linear_model.state_dict(), "log_sigma": self.log_sigma.data}, path)

    def load_model(self, path: str):
        ckpt = torch.load(path, map_location=self.device, weights_only=True)
        if self.linear_model is None:
            raise RuntimeError("Model not initialized. Train or initialize the model before loading.")
        self.linear_model.load_state_dict(ckpt["linear_state_dict"])
        self.log_sigma.data = ckpt["log_sigma"]
        self._invalidate()


class LogisticRegression(_Parametric):
    """logistIc_regression.py:11-141: logistic density with location W q + b."""

    def __init__(self, config: Dict, **kwargs):
        super().__init__(config, **kwargs)
        self._setup_model(config, **kwargs)
        self.linear_model = None
        self.log_scale = None

    def _setup_model(self, config: Dict, **kwargs):
        self.config_optimizer = config.get("optimizer", {})
        self.n_epochs = config.get("train", {}).get("n_epochs", 1000)

    def _linears(self):
        return [self.linear_model] if self.linear_model is not None else []

    def _log_scale(self):
        return self.log_scale

    def _fit(self, node_data: torch.Tensor, parents_data: torch.Tensor = None):
        """logistIc_regression.py:23-63 (intercept-only input of ones for a root)."""
        device = self.device
        if parents_data is not None:
            input_dim = parents_data.shape[0]
            queries = parents_data.transpose(0, 1).to(device).to(torch.float32)
        else:
            input_dim = 1
            queries = torch.ones((node_data.shape[0], 1), device=device).to(torch.float32)
        if self.linear_model is None:
            self.linear_model = nn.Linear(input_dim, 1).to(device).to(torch.float32)
            self.log_scale = nn.Parameter(torch.tensor(0.0, device=device))
        targets = node_data.to(device).unsqueeze(1).float()
        optimizer = config_torch_optimizer(self.linear_model, self.config_optimizer)
        loss_fn = nn.BCEWithLogitsLoss()
        bar = (tqdm(range(self.n_epochs), desc="training logistic regression...") if self.if_log
               else range(self.n_epochs))
        for _ in bar:
            optimizer.zero_grad()
            loss = loss_fn(self.linear_model(queries), targets)
            loss.backward()
            optimizer.step()
            if self.if_log:
                bar.set_postfix(loss=f"{loss.item():.4f}")
        self._invalidate()

    def _sample(self, N: int, **kwargs) -> torch.Tensor:
        """logistIc_regression.py:100-123: Bernoulli labels from sigmoid(logits)."""
        query = kwargs.get("query")
        if query is not None:
            prob = torch.sigmoid(self.linear_model(query.squeeze(-1).to(self.device)))
            return torch.bernoulli(prob.expand(prob.shape[0], N)).detach()
        prob = torch.sigmoid(self.linear_model(torch.ones((1, 1), device=self.device)))
        return torch.bernoulli(prob.expand(N)).detach()

    def save_model(self, path: str):
        torch.save({"linear_state_dict": self.linear_model.state_dict(), "log_scale": self.log_scale.data}, path)

    def load_model(self, path: str):
        ckpt = torch.load(path, map_location=self.device, weights_only=True)
        if self.linear_model is None:
            raise RuntimeError("Model not initialized. Train or initialize the model before loading.")
        self.linear_model.load_state_dict(ckpt["linear_state_dict"])
        self.log_scale.data = ckpt["log_scale"]
        self._invalidate()


class NeuralNetwork(_Parametric):
    """neural_network.py:21-165: logistic density with location mlp(q)."""

    def __init__(self, config: Dict, **kwargs):
        super().__init__(config, **kwargs)
        self._setup_model(config, **kwargs)
        self.nn_model = None
        self.log_scale = None

    def _setup_model(self, config: Dict, **kwargs):
        self.config_optimizer = config.get("optimizer", {})
        self.n_epochs = config.get("train", {}).get("n_epochs", 1000)
        config_model = config.get("model", {})
        self.hidden_dims = config_model.get("hidden_dims", [32])
        activation_name = config_model.get("activation", "tanh").lower()
        if activation_name is None:
            raise ValueError(f"Unsupported activation: {activation_name}")
        self.activation = activation_map[activation_name]()

    def _build_nn(self, input_dim: int) -> nn.Module:
        layers, cur = [], input_dim
        for h in self.hidden_dims:
            layers += [nn.Linear(cur, h), self.activation]
            cur = h
        layers.append(nn.Linear(cur, 1))
        return nn.Sequential(*layers)

    def _linears(self):
        return [m for m in self.nn_model if isinstance(m, nn.Linear)] if self.nn_model is not None else []

    def _activation_name(self):
        return _ACT_ID[type(self.activation)]

    def _log_scale(self):
        return self.log_scale

    def _fit(self, node_data: torch.Tensor, parents_data: torch.Tensor = None):
        """neural_network.py:54-93."""
        device = self.device
        if parents_data is not None:
            input_dim = parents_data.shape[0]
            queries = parents_data.transpose(0, 1).to(device).to(torch.float32)
        else:
            input_dim = 1
            queries = torch.ones((node_data.shape[0], 1), device=device).to(torch.float32)
        if self.nn_model is None:
            self.nn_model = self._build_nn(input_dim).to(device).to(torch.float32)
            self.log_scale = nn.Parameter(torch.tensor(0.0, device=device))
        targets = node_data.to(device).unsqueeze(1).float()
        optimizer = config_torch_optimizer(self.nn_model, self.config_optimizer)
        loss_fn = nn.BCEWithLogitsLoss()
        bar = (tqdm(range(self.n_epochs), desc="training neural network estimator...") if self.if_log
               else range(self.n_epochs))
        for _ in bar:
            optimizer.zero_grad()
            loss = loss_fn(self.nn_model(queries), targets)
            loss.backward()
            optimizer.step()
            if self.if_log:
                bar.set_postfix(loss=f"{loss.item():.4f}")
        self._invalidate()

    def _sample(self, N: int, **kwargs) -> torch.Tensor:
        """neural_network.py:126-147."""
        query = kwargs.get("query")
        if query is not None:
            prob = torch.sigmoid(self.nn_model(query.squeeze(-1).to(self.device)))
            return torch.bernoulli(prob.expand(prob.shape[0], N)).detach()
        prob = torch.sigmoid(self.nn_model(torch.ones((1, 1), device=self.device)))
        return torch.bernoulli(prob.expand(N)).detach()

    def save_model(self, path: str):
        torch.save({"nn_state_dict": self.nn_model.state_dict(), "log_scale": self.log_scale.data}, path)

    def load_model(self, path: str):
        ckpt = torch.load(path, map_location=self.device, weights_only=True)
        if self.nn_model is None:
            raise RuntimeError("Model not initialized. Train or initialize the model before loading.")
        self.nn_model.load_state_dict(ckpt["nn_state_dict"])
        self.log_scale.data = ckpt["log_scale"]
        self._invalidate()
