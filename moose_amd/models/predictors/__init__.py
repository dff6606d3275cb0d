"""Model zoo: secure inference for linear models, tree ensembles and neural networks
imported from ONNX (reference ``pymoose/pymoose/predictors``)."""
from moose_amd.models.predictors.base import DEFAULT_FIXED_DTYPE  # noqa: F401
from moose_amd.models.predictors.base import DEFAULT_FLOAT_DTYPE  # noqa: F401
from moose_amd.models.predictors.base import AesWrapper  # noqa: F401
from moose_amd.models.predictors.base import Predictor  # noqa: F401
from moose_amd.models.predictors.convert import from_onnx  # noqa: F401
from moose_amd.models.predictors.linear import LinearClassifier  # noqa: F401
from moose_amd.models.predictors.linear import LinearRegressor  # noqa: F401
from moose_amd.models.predictors.linear import PostTransform  # noqa: F401
from moose_amd.models.predictors.neural import Activation  # noqa: F401
from moose_amd.models.predictors.neural import MLPClassifier  # noqa: F401
from moose_amd.models.predictors.neural import MLPRegressor  # noqa: F401
from moose_amd.models.predictors.neural import NeuralNetwork  # noqa: F401
from moose_amd.models.predictors.onnx_proto import load_model  # noqa: F401
from moose_amd.models.predictors.trees import TreeEnsembleClassifier  # noqa: F401
from moose_amd.models.predictors.trees import TreeEnsembleRegressor  # noqa: F401
