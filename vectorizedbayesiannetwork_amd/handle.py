"""Per-node CPD inspector with the reference ``CPDHandle`` surface
(reference ``vbn/core/cpd_handle.py``), backed by single-node GPU walks.

``VBN.cpd(node)`` / ``get_cpd`` / ``get_cpds`` return these.  ``sample`` / ``log_prob`` /
``pdf`` / ``forward`` run the node's CPD on the MI355X (:mod:`.cpd`); ``conditional`` returns
the reference's formats (``cpd_handle.py:348-404``):

* ``normal_params``   -- gaussian_nn, linear_gaussian: ``mean`` / ``std`` [B, 1 | S, D]
  (walk role PARAMS);
* ``mixture_params``  -- mdn: ``weights`` = softmax(logits) [B, 1, K], ``loc`` / ``scale``
  [B, 1, K, D] (PARAMS);
* ``categorical_probs`` -- softmax_nn: ``probs`` [B, 1, D, C], ``k``, ``support``
  (``_sample_values``) (PARAMS);
* ``empirical_samples`` -- kde: ``n_samples`` GPU draws with their mean / std.

As in the reference, tensors in the returned dicts go through ``to_serializable`` (nested
lists up to 2048 elements, a shape summary beyond); :meth:`CPDHandle.conditional_tensors`
returns the same fields as device tensors.
"""
from __future__ import annotations

from typing import Any, Dict, Optional

import torch

from . import cpd as C
from .model import CPDRecord

__all__ = ["CPDHandle", "to_serializable"]

_CLASS_NAME = {"gaussian_nn": "GaussianNNCPD", "linear_gaussian": "LinearGaussianCPD", "mdn": "MDNCPD",
               "kde": "KDECPD", "softmax_nn": "SoftmaxNNCPD"}


def to_serializable(obj, *, max_tensor_elems: int = 2048):
    """reference core/utils.py:102-128"""
    if obj is None or isinstance(obj, (str, int, float, bool)):
        return obj
    if isinstance(obj, (torch.device, torch.dtype)):
        return str(obj)
    if isinstance(obj, torch.Tensor):
        t = obj.detach()
        if int(t.numel()) <= max_tensor_elems:
            return t.cpu().tolist()
        return {"type": "tensor", "shape": list(t.shape), "dtype": str(t.dtype), "device": str(t.device),
                "numel": int(t.numel())}
    if isinstance(obj, dict):
        return {str(k): to_serializable(v, max_tensor_elems=max_tensor_elems) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [to_serializable(v, max_tensor_elems=max_tensor_elems) for v in obj]
    return str(obj)


class CPDHandle:
    """reference core/cpd_handle.py:129-428 (same properties, argument forms and errors)."""

    def __init__(self, vbn, node: str) -> None:
        if node not in vbn.nodes:
            raise ValueError(f"Unknown node '{node}'.")
        self._vbn = vbn
        self._node = node
        self._rec: CPDRecord = vbn.model.cpds[node]
        self._parents = list(vbn.dag.parents(node))

    # ---- description ---------------------------------------------------------------------
    @property
    def node(self) -> str:
        return self._node

    name = node

    @property
    def cpd(self) -> CPDRecord:
        return self._rec

    @property
    def cpd_name(self) -> str:
        return self._rec.kind

    @property
    def cpd_type(self) -> str:
        return _CLASS_NAME[self._rec.kind]

    @property
    def parents(self):
        return list(self._parents)

    @property
    def is_fitted(self) -> bool:
        st = self._rec.state
        if self._rec.kind == "kde":
            return bool(self._rec.extra and self._rec.extra.get("targets") is not None)
        for flag in ("_bins_ready", "_stats_ready"):
            if flag in st:
                return bool(st[flag])
        return bool(st)

    @property
    def device(self) -> torch.device:
        return self._vbn.device

    @property
    def x_dim(self) -> int:
        return int(self._rec.output_dim)

    output_dim = x_dim

    @property
    def parents_dim(self) -> int:
        return int(self._rec.input_dim)

    input_dim = parents_dim

    def summary(self) -> dict:
        return {"node": self.node, "parents": self.parents, "cpd_name": self.cpd_name,
                "cpd_type": self.cpd_type, "input_dim": self.input_dim, "output_dim": self.output_dim,
                "device": str(self.device), "is_fitted": self.is_fitted}

    def export_config(self) -> dict:
        return {"node": self.node, "parents": self.parents, "cpd_name": self.cpd_name,
                "cpd_type": self.cpd_type, "init_kwargs": to_serializable(dict(self._rec.hparams)),
                "extra_state": to_serializable(self._rec.extra)}

    def state_dict(self) -> dict:
        return dict(self._rec.state)

    # ---- inputs (cpd_handle.py:203-261) -------------------------------------------------------
    def _as_tensor(self, v) -> torch.Tensor:
        t = v if isinstance(v, torch.Tensor) else torch.as_tensor(v)
        return t.to(device=self._vbn.device, dtype=torch.float32)

    def _parents_tensor(self, parents) -> Optional[torch.Tensor]:
        if self.parents_dim == 0:
            if parents is None or (isinstance(parents, dict) and not parents):
                return None
            if isinstance(parents, torch.Tensor):
                t = self._as_tensor(parents)
                if t.dim() == 2 and t.shape[-1] == 0:
                    return None
            raise ValueError(f"Node '{self._node}' has no parents.")
        if parents is None:
            raise ValueError(f"Parents required for node '{self._node}'.")
        if isinstance(parents, dict):
            ts = []
            for p in self._parents:
                if p not in parents:
                    raise ValueError(f"Missing parent '{p}' for node '{self._node}'.")
                t = self._as_tensor(parents[p])
                ts.append(t.unsqueeze(-1) if t.dim() == 1 else t)
            t = torch.cat(ts, dim=-1)
            if t.shape[-1] != self.parents_dim:
                raise ValueError(f"Expected parents_dim {self.parents_dim}, got {t.shape[-1]}")
            return t
        if isinstance(parents, torch.Tensor):
            t = self._as_tensor(parents)
            if t.dim() == 1:
                t = t.unsqueeze(-1)
            if t.dim() not in (2, 3):
                raise ValueError(f"Expected parents with 2D or 3D shape, got {tuple(t.shape)}")
            if t.shape[-1] != self.parents_dim:
                raise ValueError(f"Expected parents_dim {self.parents_dim}, got {t.shape[-1]}")
            return t
        raise TypeError("parents must be a tensor or dict")

    def _x_tensor(self, x) -> torch.Tensor:
        t = self._as_tensor(x)
        if t.dim() == 1:
            t = t.unsqueeze(-1)
        if t.dim() not in (2, 3):
            raise ValueError(f"Expected x with 2D or 3D shape, got {tuple(t.shape)}")
        return t

    # ---- evaluation on the GPU ------------------------------------------------------------
    def sample(self, parents, n_samples: int, **kw) -> torch.Tensor:
        return C.cpd_sample(self._vbn, self._node, self._parents_tensor(parents), int(n_samples), **kw).detach()

    def log_prob(self, x, parents) -> torch.Tensor:
        return C.cpd_log_prob(self._vbn, self._node, self._x_tensor(x), self._parents_tensor(parents)).detach()

    def pdf(self, x, parents) -> torch.Tensor:
        return torch.exp(self.log_prob(x, parents))

    def forward(self, parents, n_samples: int, **kw) -> C.CPDOutput:
        out = C.cpd_forward(self._vbn, self._node, self._parents_tensor(parents), int(n_samples), **kw)
        return C.CPDOutput(samples=out.samples.detach(), log_prob=out.log_prob.detach(), pdf=out.pdf.detach())

    def conditional_samples(self, parents, n_samples: int = 1024) -> torch.Tensor:
        return self.sample(parents, n_samples)

    def conditional_log_prob(self, x, parents) -> torch.Tensor:
        return self.log_prob(x, parents)

    def conditional_pdf(self, x, parents) -> torch.Tensor:
        return self.pdf(x, parents)

    def conditional_tensors(self, parents, *, n_samples: int = 1024, **kw) -> Dict[str, Any]:
        """The fields of :meth:`conditional` as device tensors (no host copies); ``kw``
        (``seed``, injected draws) goes to the kde sampler."""
        pt = self._parents_tensor(parents)
        kind, D = self._rec.kind, self.output_dim
        if kind == "kde":
            s = self.sample(pt, n_samples, **kw)
            return {"format": "empirical_samples", "samples": s, "mean": s.mean(dim=1),
                    "std": s.std(dim=1, unbiased=False), "n_samples": int(n_samples)}
        prm = C.cpd_params(self._vbn, self._node, pt)                  # [B, 1 | S, W]
        b, s = prm.shape[0], prm.shape[1]
        if kind in ("gaussian_nn", "linear_gaussian"):
            return {"format": "normal_params", "mean": prm[..., :D], "std": prm[..., D:2 * D]}
        if kind == "mdn":
            k = int(self._rec.hp("n_components"))
            return {"format": "mixture_params", "weights": prm[..., :k],
                    "loc": prm[..., k:k + k * D].reshape(b, s, k, D),
                    "scale": prm[..., k + k * D:].reshape(b, s, k, D)}
        c = int(self._rec.hp("n_classes"))
        return {"format": "categorical_probs", "probs": prm.reshape(b, s, D, c), "k": c,
                "support": self._rec.state["_sample_values"].to(self._vbn.device)}

    def conditional(self, parents, *, n_samples: int = 1024) -> dict:
        """reference cpd_handle.py:348-404"""
        pt = self._parents_tensor(parents)
        base = {"node": self.node, "parents": self.parents, "cpd_name": self.cpd_name,
                "cpd_type": self.cpd_type, "input_dim": self.input_dim, "output_dim": self.output_dim,
                "conditioning": to_serializable(pt)}
        out = self.conditional_tensors(pt, n_samples=n_samples)
        return {**base, **{k: (v if k in ("format", "k", "n_samples") else to_serializable(v))
                           for k, v in out.items()}}

    def conditional_mean_std(self, parents, n_samples: int = 1024) -> dict:
        """reference cpd_handle.py:415-428"""
        if self._rec.kind in ("gaussian_nn", "linear_gaussian"):
            t = self.conditional_tensors(parents)
            return {"format": "normal_params", "mean": t["mean"], "std": t["std"]}
        s = self.sample(parents, n_samples)
        return {"format": "empirical_samples", "mean": s.mean(dim=1), "std": s.std(dim=1, unbiased=False)}
