# Namespace-friendly: when the reference's `flex` package is also on sys.path, its other
# subpackages (ionic_bond, tools, federated_*) stay importable next to this paillier engine.
from pkgutil import extend_path

__path__ = extend_path(__path__, __name__)
