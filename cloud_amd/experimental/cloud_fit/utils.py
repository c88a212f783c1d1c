"""Strategy-name registry (reference ``cloud_fit/utils.py:19-39``): the same
``distribution_strategy=`` strings select the MI355X-native strategies."""
from ...parallel import strategy as S

SUPPORTED_DISTRIBUTION_STRATEGIES = {
    S.MultiWorkerMirroredStrategy.__name__: S.MultiWorkerMirroredStrategy,
    S.MirroredStrategy.__name__: S.MirroredStrategy,
}
MULTI_WORKER_MIRRORED_STRATEGY_NAME = S.MultiWorkerMirroredStrategy.__name__
MIRRORED_STRATEGY_NAME = S.MirroredStrategy.__name__


def is_tf_v1():
    return False
