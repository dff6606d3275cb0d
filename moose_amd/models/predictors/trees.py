"""Tree ensembles (random forests, gradient-boosted trees) for regression and
classification.

Parity: reference ``pymoose/pymoose/predictors/tree_ensemble.py`` (same ONNX
``TreeEnsembleRegressor``/``TreeEnsembleClassifier`` semantics and post transforms).

Evaluation is restructured for the MI355X instead of the reference's recursive
``mux`` per node:

1. every split of every tree is evaluated in ONE batched secure comparison
   (``less`` over a [batch, n_splits] gather of feature columns vs public thresholds);
2. leaf-reaching indicators are propagated top-down one tree *level* at a time for all
   trees at once: ``left = mux(split, parent, 0)``, ``right = parent - left`` -- one
   batched multiplication per level;
3. the prediction is one public-weight matmul ``indicators[batch, leaves] @ W[leaves,
   outputs]``.

Round count is ``comparison + depth x (mux)`` regardless of the number of trees; the
reference's count is the same depth but with one protocol invocation per node.
"""
from __future__ import annotations

import json
from dataclasses import dataclass
from typing import Dict
from typing import List
from typing import Tuple

import numpy as np

import moose_amd as pm
from moose_amd.models.predictors.base import DEFAULT_FIXED_DTYPE
from moose_amd.models.predictors.base import Predictor
from moose_amd.models.predictors.base import find_attribute
from moose_amd.models.predictors.base import find_node
from moose_amd.models.predictors.base import load_onnx
from moose_amd.models.predictors.base import n_input_features


@dataclass
class Tree:
    """node id -> (feature, threshold, left id, right id) for splits; leaves map to
    {output column: weight}.  ``x[feature] < threshold`` goes left."""

    root: int
    splits: Dict[int, Tuple[int, float, int, int]]
    leaves: Dict[int, Dict[int, float]]

    def levels(self):
        """Split nodes grouped by depth (root = depth 0)."""
        out, frontier = [], [self.root]
        while frontier:
            lvl = [n for n in frontier if n in self.splits]
            if not lvl:
                break
            out.append(lvl)
            nxt = []
            for n in lvl:
                _, _, le, ri = self.splits[n]
                nxt += [le, ri]
            frontier = nxt
        return out


def _build_trees(treeids, nodeids, featureids, values, trues, falses, modes,
                 w_treeids, w_nodeids, w_ids, w_weights, collapse_outputs=False) -> List[Tree]:
    splits: Dict[int, Dict[int, tuple]] = {}
    leaves: Dict[int, Dict[int, Dict[int, float]]] = {}
    children = {}
    for i, t in enumerate(treeids):
        n = nodeids[i]
        mode = modes[i] if modes else b"BRANCH_LT"
        if (mode == b"LEAF") or (trues[i] == 0 and falses[i] == 0):
            leaves.setdefault(t, {}).setdefault(n, {})
        else:
            splits.setdefault(t, {})[n] = (int(featureids[i]), float(values[i]), int(trues[i]),
                                           int(falses[i]))
            children.setdefault(t, set()).update((trues[i], falses[i]))
    for i, t in enumerate(w_treeids):
        col = 0 if collapse_outputs else int(w_ids[i])
        d = leaves.setdefault(t, {}).setdefault(int(w_nodeids[i]), {})
        d[col] = d.get(col, 0.0) + float(w_weights[i])
    trees = []
    for t in sorted(set(treeids)):
        ids = set(splits.get(t, {})) | set(leaves.get(t, {}))
        roots = sorted(ids - children.get(t, set()))
        trees.append(Tree(roots[0], splits.get(t, {}), leaves.get(t, {})))
    return trees


class TreeEnsemble(Predictor):
    def __init__(self, trees: List[Tree], n_features: int, n_outputs: int,
                 base_score: float = 0.0):
        super().__init__()
        self.trees = trees
        self.n_features = n_features
        self.n_outputs = n_outputs
        self.base_score = base_score
        if trees:
            used = [f for t in trees for (f, _, _, _) in t.splits.values()]
            if used and max(used) >= n_features:
                raise ValueError(f"split feature index {max(used)} >= {n_features} features")

    # -- secure evaluation --------------------------------------------------------------
    def constant_leaves(self) -> np.ndarray:
        """Contribution of single-leaf trees (no split to evaluate)."""
        row = np.zeros(self.n_outputs)
        for t in self.trees:
            if t.root in t.leaves:
                for c, w in t.leaves[t.root].items():
                    row[c] += w
        return row

    def scores(self, x, fixedpoint_dtype=DEFAULT_FIXED_DTYPE):
        """[batch, n_outputs] raw ensemble scores (before base score / transform)."""
        split_keys, feats, thr = [], [], []
        level_nodes: List[List[Tuple[int, int]]] = []
        for ti, t in enumerate(self.trees):
            for d, lvl in enumerate(t.levels()):
                while len(level_nodes) <= d:
                    level_nodes.append([])
                level_nodes[d] += [(ti, n) for n in lvl]
        col = {}
        for lvl in level_nodes:
            for (ti, n) in lvl:
                f, v, _, _ = self.trees[ti].splits[n]
                col[(ti, n)] = len(split_keys)
                split_keys.append((ti, n))
                feats.append(f)
                thr.append(v)
        ind = {}  # (tree, node) -> (indicator block of its level, column)
        leaf_exprs = []
        if split_keys:
            xs = pm.concatenate([pm.expand_dims(pm.index_axis(x, axis=1, index=f), 1)
                                 for f in feats], axis=1)
            t_c = self.fixedpoint_constant(np.asarray(thr, dtype=np.float64), plc=self.mirrored,
                                           dtype=fixedpoint_dtype)
            sel = pm.less(xs, t_c)  # ONE comparison for every split of every tree
            for d, lvl in enumerate(level_nodes):
                s_d = pm.concatenate([pm.expand_dims(pm.index_axis(sel, axis=1,
                                                                   index=col[k]), 1)
                                      for k in lvl], axis=1)
                if d == 0:
                    ones = pm.ones(pm.shape(s_d), dtype=pm.float64, placement=self.mirrored)
                    p_d = pm.cast(ones, dtype=fixedpoint_dtype, placement=self.mirrored)
                else:
                    p_d = pm.concatenate([pm.expand_dims(pm.index_axis(ind[k][0], axis=1,
                                                                       index=ind[k][1]), 1)
                                          for k in lvl], axis=1)
                zeros = pm.zeros(pm.shape(s_d), dtype=pm.float64, placement=self.mirrored)
                z_d = pm.cast(zeros, dtype=fixedpoint_dtype, placement=self.mirrored)
                left = pm.mux(s_d, p_d, z_d)
                right = pm.sub(p_d, left)
                for j, (ti, n) in enumerate(lvl):
                    _, _, le, ri = self.trees[ti].splits[n]
                    ind[(ti, le)] = (left, j)
                    ind[(ti, ri)] = (right, j)
        w_rows = []
        for ti, t in enumerate(self.trees):
            for n, wd in sorted(t.leaves.items()):
                if (ti, n) not in ind:
                    continue  # a single-leaf tree (see constant_leaves) or unreachable
                row = np.zeros(self.n_outputs)
                for c, w in wd.items():
                    row[c] += w
                w_rows.append(row)
                e, j = ind[(ti, n)]
                leaf_exprs.append(pm.expand_dims(pm.index_axis(e, axis=1, index=j), 1))
        if not leaf_exprs:
            raise ValueError("tree ensemble without reachable leaves")
        indicators = pm.concatenate(leaf_exprs, axis=1)  # [batch, n_leaves]
        w = self.fixedpoint_constant(np.asarray(w_rows), plc=self.mirrored, dtype=fixedpoint_dtype)
        return pm.dot(indicators, w)

    def _with_base(self, y, fixedpoint_dtype):
        base = np.full(self.n_outputs, float(self.base_score)) + self.constant_leaves()
        b = self.fixedpoint_constant(base, plc=self.mirrored, dtype=fixedpoint_dtype)
        return pm.add(y, b)


class TreeEnsembleRegressor(TreeEnsemble):
    def predict(self, x, fixedpoint_dtype=DEFAULT_FIXED_DTYPE):
        y = self._with_base(self.scores(x, fixedpoint_dtype), fixedpoint_dtype)
        if self.n_outputs == 1:
            return pm.index_axis(y, axis=1, index=0)
        return y

    @classmethod
    def from_onnx(cls, model):
        model = load_onnx(model)
        node, base, trees_args, nf = _onnx_forest(model, "TreeEnsembleRegressor")
        a = {n: find_attribute(node, n, enforce=False) for n in
             ("target_treeids", "target_nodeids", "target_ids", "target_weights", "n_targets")}
        n_targets = int(a["n_targets"].i) if a["n_targets"] is not None else 1
        ids = a["target_ids"].ints if a["target_ids"] is not None else [0] * len(a["target_treeids"].ints)
        trees = _build_trees(*trees_args, a["target_treeids"].ints, a["target_nodeids"].ints,
                             ids, a["target_weights"].floats)
        return cls(trees, nf, n_targets, base)

    @classmethod
    def from_json(cls, forest_json):
        """XGBoost JSON model dump (``Booster.save_model("m.json")``)."""
        if isinstance(forest_json, (str, bytes)):
            forest_json = json.loads(forest_json)
        learner = forest_json["learner"]
        booster = learner["gradient_booster"]["model"]
        nf = int(learner["learner_model_param"]["num_feature"])
        base = float(learner["learner_model_param"]["base_score"])
        trees = []
        for tj in booster["trees"]:
            left, right = tj["left_children"], tj["right_children"]
            splits, leaves = {}, {}
            for n in range(len(left)):
                if left[n] == -1:
                    leaves[n] = {0: float(tj["base_weights"][n])}
                else:
                    splits[n] = (int(tj["split_indices"][n]), float(tj["split_conditions"][n]),
                                 int(left[n]), int(right[n]))
            trees.append(Tree(0, splits, leaves))
        return cls(trees, nf, 1, base)


class TreeEnsembleClassifier(TreeEnsemble):
    def __init__(self, trees, n_features, n_classes, base_score=0.0, transform_output=False):
        self.n_classes = n_classes
        self.transform_output = transform_output
        super().__init__(trees, n_features, 1 if n_classes == 2 else n_classes, base_score)

    def predict(self, x, fixedpoint_dtype=DEFAULT_FIXED_DTYPE):
        y = self._with_base(self.scores(x, fixedpoint_dtype), fixedpoint_dtype)
        if self.n_classes == 2:
            pos = pm.sigmoid(y) if self.transform_output else y  # [batch, 1]
            one = self.fixedpoint_constant(1.0, plc=self.mirrored, dtype=fixedpoint_dtype)
            return pm.concatenate([pm.sub(one, pos), pos], axis=1)
        if self.transform_output:
            return pm.softmax(y, axis=1, upmost_index=self.n_classes)
        return y

    @classmethod
    def from_onnx(cls, model):
        model = load_onnx(model)
        node, base, trees_args, nf = _onnx_forest(model, "TreeEnsembleClassifier")
        labels = (find_attribute(node, "classlabels_int64s", enforce=False)
                  or find_attribute(node, "classlabels_strings", enforce=False))
        n_classes = len(labels.ints) or len(labels.strings)
        a = {n: find_attribute(node, n) for n in
             ("class_treeids", "class_nodeids", "class_ids", "class_weights")}
        # binary models: every leaf weight feeds the single (positive-class) score, as in
        # the reference (tree_ensemble.py _maybe_sigmoid)
        trees = _build_trees(*trees_args, a["class_treeids"].ints, a["class_nodeids"].ints,
                             a["class_ids"].ints, a["class_weights"].floats,
                             collapse_outputs=(n_classes == 2))
        pt = find_attribute(node, "post_transform").s.decode()
        return cls(trees, nf, n_classes, base, transform_output=(pt != "NONE"))


def _onnx_forest(model, op_type):
    node = find_node(model, op_type, enforce=False)
    if node is None:
        raise ValueError(f"Incompatible ONNX graph provided: graph must contain a {op_type} "
                         "operator.")

    def ints(n):
        return list(find_attribute(node, n).ints)

    modes_a = find_attribute(node, "nodes_modes", enforce=False)
    modes = list(modes_a.strings) if modes_a is not None else None
    args = (ints("nodes_treeids"), ints("nodes_nodeids"), ints("nodes_featureids"),
            list(find_attribute(node, "nodes_values").floats), ints("nodes_truenodeids"),
            ints("nodes_falsenodeids"), modes)
    nf = n_input_features(model)
    bv = find_attribute(node, "base_values", enforce=False)
    # the reference adds base_values[0] to every output (tree_ensemble.py _onnx_base)
    base = float(bv.floats[0]) if bv is not None and bv.floats else 0.0
    return node, base, args, nf

