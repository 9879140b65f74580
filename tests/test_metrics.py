import numpy as np
import pytest
from sklearn.metrics import accuracy_score, confusion_matrix, f1_score, precision_score, recall_score

from mtl_das_pytorch_amd.utils.metrics import (confusion_from_lists, mae_from_confusion, metrics_from_confusion,
                                               sklearn_confusion)


@pytest.mark.parametrize("n,seed", [(16, 0), (2, 1), (16, 2)])
def test_metrics_match_sklearn(n, seed):
    rng = np.random.RandomState(seed)
    y = rng.randint(0, n, 200)
    p = np.where(rng.rand(200) < 0.6, y, rng.randint(0, n - 2 if n > 2 else n, 200))
    if n == 16:
        y[y == 15] = 14  # make one class absent: sklearn's label set shrinks
    cm = confusion_from_lists(y, p, n)
    m = metrics_from_confusion(cm)
    assert np.array_equal(sklearn_confusion(cm), confusion_matrix(y, p))
    assert m["accuracy"] == pytest.approx(accuracy_score(y, p))
    np.testing.assert_allclose(m["f1_per_class"], f1_score(y, p, average=None, zero_division=0), rtol=1e-12)
    assert m["f1_weighted"] == pytest.approx(f1_score(y, p, average="weighted", zero_division=0))
    assert m["precision_weighted"] == pytest.approx(precision_score(y, p, average="weighted", zero_division=0))
    assert m["recall_weighted"] == pytest.approx(recall_score(y, p, average="weighted", zero_division=0))


def test_mae():
    cm = np.zeros((16, 16), int)
    cm[3, 5] = 2
    cm[7, 7] = 2
    assert mae_from_confusion(cm) == 1.0
