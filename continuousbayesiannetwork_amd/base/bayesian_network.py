"""BayesianNetwork: DAG + per-node estimators + batched inference.

Mirrors cbn/base/bayesian_network.py (constructor signature and validation,
graph helpers, ``update_knowledge``, ``get_pdf``, ``infer``,
``benchmarking_df``).  ``infer`` returns the reference's numbers
(bayesian_network.py:208-305: product over the target's ancestors of each
factor's mean over its parent axes, divided by the global max) computed by the
HIP engine in ``inference/engine.py``.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Tuple

import networkx as nx
import numpy as np
import pandas as pd
import torch
from tqdm import tqdm

from . import BASE_MAX_CARDINALITY, KEY_MAX_CARDINALITY_FOR_DISCRETE
from .node import Node
from ..utils import choose_inference_obj


class BayesianNetwork:
    def __init__(self, dag: nx.DiGraph, data: pd.DataFrame, parameters_learning_config: Dict,
                 inference_config: Dict, **kwargs):
        if not nx.is_directed_acyclic_graph(dag):
            raise ValueError("The provided graph is not a directed acyclic graph (DAG).")
        self.initial_dag = dag
        self.column_mapping = {node: i for i, node in enumerate(self.initial_dag.nodes)}
        self.device = "cuda" if torch.cuda.is_available() else "cpu"
        kwargs["device"] = self.device if "device" not in kwargs else kwargs["device"]
        self.device = kwargs["device"]
        self.min_tolerance = kwargs.get("min_tolerance", 1e-10)
        self.uncertainty = kwargs.get("uncertainty", 1e-10)
        self.max_cardinality_for_discrete_domain = kwargs.get(KEY_MAX_CARDINALITY_FOR_DISCRETE, BASE_MAX_CARDINALITY)
        self.log = kwargs.get("log", False)
        self.nodes_obj = None
        self._kwargs = kwargs
        from ..inference.engine import InferenceEngine

        self.engine = InferenceEngine(self)
        self._setup_parameters_learning(data, parameters_learning_config, **kwargs)
        self._setup_inference(inference_config)

    def _setup_parameters_learning(self, data: pd.DataFrame, config: Dict, **kwargs):
        estimator_name = config["estimator_name"]
        self.nodes_obj = {
            node: Node(node, estimator_name, config, self.get_parents(self.initial_dag, node), **kwargs)
            for node in self.initial_dag.nodes
        }
        nodes = self.initial_dag.nodes
        pbar = tqdm(nodes, total=len(nodes), desc="training probability estimator...") if self.log else nodes
        self._train(data, pbar)

    def _setup_inference(self, config: Dict):
        self.inference_obj_name = config["inference_obj"]
        self.inference_obj = choose_inference_obj(self.inference_obj_name, config, bn=self, device=self.device)

    def save_model(self, path: str):
        for node in self.nodes_obj:
            self.nodes_obj[node].save_node(path)

    @staticmethod
    def get_nodes(dag: nx.DiGraph):
        return sorted(list(dag.nodes))

    def _name(self, node):
        return next((k for k, v in self.column_mapping.items() if v == node), None)

    def get_ancestors(self, dag: nx.DiGraph, node):
        """bayesian_network.py:86-102: ancestors in topological order (farthest first)."""
        if isinstance(node, str):
            ancestors = nx.ancestors(dag, node)
        elif isinstance(node, int):
            name = self._name(node)
            if name is None:
                return set()
            ancestors = nx.ancestors(dag, name)
        else:
            raise ValueError(f"{node} type not supported.")
        order = list(nx.topological_sort(dag.subgraph(ancestors | {node})))
        order.remove(node)
        return order

    def get_parents(self, dag: nx.DiGraph, node):
        if isinstance(node, str):
            return sorted(list(dag.predecessors(node)))
        elif isinstance(node, int):
            return sorted(list(dag.predecessors(self._name(node))))
        raise ValueError(f"{node} type not supported.")

    def get_children(self, dag: nx.DiGraph, node):
        if isinstance(node, str):
            return sorted(list(dag.successors(node)))
        elif isinstance(node, int):
            return sorted(list(dag.successors(self._name(node))))
        raise ValueError(f"{node} type not supported.")

    def update_knowledge(self, data: pd.DataFrame):
        nodes = self.initial_dag.nodes
        pbar = tqdm(nodes, total=len(nodes), desc="updating probability estimator...") if self.log else nodes
        self._train(data, pbar)

    def _train(self, data: pd.DataFrame, pbar: Iterable):
        """bayesian_network.py:138-160."""
        if self.engine is not None:
            self.engine.invalidate()
        is_tqdm = isinstance(pbar, tqdm)
        for node in pbar:
            if is_tqdm:
                pbar.set_postfix(updating_node=f"{node}")
            node_data = torch.tensor(np.array(data[node].values.tolist(), dtype=np.float32), device=self.device)
            node_parents = self.get_parents(self.initial_dag, node)
            parents_data = (
                torch.tensor(np.array(data[node_parents].values.tolist(), dtype=np.float32), device=self.device).T
                if node_parents else None)
            self.nodes_obj[node].fit(node_data, parents_data)

    @staticmethod
    def get_structure(dag: nx.DiGraph):
        return {node: list(dag.predecessors(node)) for node in nx.topological_sort(dag)}

    def get_pdf(self, target_node: str, evidence: Dict, N_max: int = 1024
                ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """bayesian_network.py:176-206: the target's factor via Node.get_prob."""
        parents = self.get_parents(self.initial_dag, target_node)
        query = {f: v for f, v in evidence.items() if f in parents}
        return self.nodes_obj[target_node].get_prob(query, N_max)

    def infer(self, target_node: str, evidence: Dict[str, torch.Tensor] = None, do: List[str] = None,
              N_max: int = 16, plot_prob=False):
        """bayesian_network.py:208-305.

        :param evidence: {node: tensor [n_queries, 1]}
        :return: (pdf [n_queries, N_max] normalised by its global max,
                  target domain [n_queries or 1, N_max])
        """
        # `do` is accepted and ignored, as in the reference (bayesian_network.py:228-232)
        out_pdf, target_node_domains = self.engine.infer(target_node, evidence, N_max)
        if plot_prob:
            self.plot_prob(out_pdf, target_node_domains, target_node)
        return out_pdf, target_node_domains

    @staticmethod
    def plot_prob(pdf, domain, target_node: str):
        assert pdf.shape == domain.shape, "pdf and domain must have same shape."
        import matplotlib.pyplot as plt

        pdf_np, dom_np = pdf.cpu().numpy(), domain.cpu().numpy()
        plt.figure(dpi=500)
        for q in range(pdf_np.shape[0]):
            plt.plot(dom_np[q], pdf_np[q], label=f"query {q}")
        plt.xlabel(f"{target_node} domain")
        plt.ylabel("PDF")
        plt.xticks(dom_np[0])
        plt.legend(loc="best")
        plt.grid(True)
        plt.show()

    def benchmarking_df(self, data: pd.DataFrame, target_feature: str, batch_size: int = 128, **kwargs) -> np.ndarray:
        """bayesian_network.py:329-373: argmax prediction of the target per row."""
        values = {f: torch.tensor(data[f].values, device="cpu") for f in data.columns if f != target_feature}
        pred = np.zeros((len(data),))
        bar = tqdm(total=len(data), desc="benchmarking df cbn...")
        for n in range(0, len(data), batch_size):
            evidence = {f: values[f][n:n + batch_size].unsqueeze(-1).to(self.device)
                        for f in data.columns if f != target_feature}
            probs, domain = self.infer(target_feature, evidence, plot_prob=False, N_max=16)
            idx = torch.argmax(probs, dim=1, keepdim=True)
            pred[n:n + batch_size] = torch.gather(domain, dim=1, index=idx).squeeze(1).cpu().numpy()
            bar.update(min(n + batch_size, len(data)) - n)
        return pred
