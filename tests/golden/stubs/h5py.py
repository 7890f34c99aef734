"""Stand-in for h5py used ONLY when running the reference scripts for golden vectors:
datasets written through ``File(path,'w').create_dataset`` land in ``path + '.npz'``;
``File(path,'r')[name]`` reads them back as numpy arrays."""
import numpy as np


class File:
    def __init__(self, path, mode="r"):
        self.path, self.mode, self.data = path, mode, {}
        if mode == "r":
            with np.load(path + ".npz") as z:
                self.data = {k: z[k] for k in z.files}

    def create_dataset(self, name, data):
        self.data[name] = np.asarray(data)

    def __getitem__(self, name):
        return self.data[name]

    def close(self):
        if self.mode == "w":
            np.savez(self.path + ".npz", **self.data)

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
