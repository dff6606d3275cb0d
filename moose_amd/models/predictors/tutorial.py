"""The reference's private-inference tutorial model (BASELINE config 4).

``/root/reference/tutorials/ml-inference-with-onnx.ipynb``: a scikit-learn
LogisticRegression trained on ``make_classification(n_samples=1000, n_features=10,
n_classes=2, random_state=5)`` with an 80/20 split (``random_state=5``), exported to ONNX
and loaded with ``predictors.from_onnx``; the 200 test rows are secret-shared from alice,
scored on the replicated placement (public weights, secure sigmoid) and the class
probabilities are opened to bob.

The ONNX graph is the one skl2onnx emits for this model (a LinearClassifier with rows
(-w, w) and a LOGISTIC post-transform), written by our own protobuf writer
(``onnx_proto``): ``onnx``/``skl2onnx`` are not importable here.  The notebook publishes no
timing, so latency parity is unpinned; accuracy is checked against sklearn's
``predict_proba``.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class TutorialModel:
    computation: object      # AbstractComputation (argument "x" on alice)
    x_test: np.ndarray       # (200, 10) float64
    proba: np.ndarray        # sklearn predict_proba(x_test), (200, 2)
    dtype: object            # fixed-point dtype the predictor runs at


def logistic_regression_tutorial(ring: int = 128) -> TutorialModel:
    """Build the tutorial's model.  Z_2^128 runs pymoose's DEFAULT_FIXED_DTYPE fixed(24, 40);
    Z_2^64 the reference's canonical Fixed64 precision fixed(14, 23)
    (``moose/src/replicated/input.rs:91-92``)."""
    from sklearn.datasets import make_classification
    from sklearn.linear_model import LogisticRegression
    from sklearn.model_selection import train_test_split

    import moose_amd as pm
    from moose_amd.models import predictors
    from moose_amd.models.predictors import onnx_proto

    X, y = make_classification(n_samples=1000, n_features=10, n_classes=2, random_state=5)
    X_train, X_test, y_train, _ = train_test_split(X, y, test_size=0.2, random_state=5)
    lg = LogisticRegression().fit(X_train, y_train)
    onnx_bytes = onnx_proto.sklearn_logistic_regression_model(lg.coef_, lg.intercept_, 10)
    model = predictors.from_onnx(onnx_bytes)
    dtype = predictors.DEFAULT_FIXED_DTYPE if ring == 128 else pm.fixed(14, 23)
    return TutorialModel(model.predictor_factory(dtype), X_test, lg.predict_proba(X_test),
                         dtype)
