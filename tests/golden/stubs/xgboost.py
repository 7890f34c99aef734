"""Stand-in for xgboost used ONLY to capture the feature matrices predict.py builds."""
import numpy as np

CAPTURED = []


class DMatrix:
    def __init__(self, data):
        self.data = np.asarray(data)
        CAPTURED.append(self.data)
        np.save(f"captured_dmatrix_{len(CAPTURED) - 1}.npy", self.data)


class Booster:
    def __init__(self, params=None):
        pass

    def load_model(self, path):
        pass

    def predict(self, d):
        return np.zeros(d.data.shape[0])
