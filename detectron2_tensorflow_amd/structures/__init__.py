"""Box containers of lib/structures (box_list.py:7-264, image_list.py:7-101).

Boxes are [ymin, xmin, ymax, xmax] in absolute pixels.  Dense BoxLists carry
fixed-size padded tensors plus an ``is_valid`` field (no host synchronisation
to learn their length); SparseBoxList keeps (image, slot) indices into such a
dense layout, image-major, as tf.where produces them.
"""
import torch


class BoxList:
    def __init__(self, boxes):
        if boxes.shape[-1] != 4:
            raise ValueError("Invalid dimensions for box data.")
        if boxes.dtype != torch.float32:
            raise ValueError("Invalid tensor type: should be float32")
        self.data = {"boxes": boxes}
        self.trackings = {}

    @property
    def boxes(self):
        return self.data["boxes"]

    def add_field(self, field, value):
        self.data[field] = value

    def has_field(self, field):
        return field in self.data

    def get_field(self, field):
        if field not in self.data:
            raise ValueError(f"field {field} does not exist")
        return self.data[field]

    def set_field(self, field, value):
        if field not in self.data:
            raise ValueError(f"field {field} does not exist")
        self.data[field] = value

    def get_all_fields(self):
        return list(self.data)

    def get_extra_fields(self):
        return [k for k in self.data if k != "boxes"]

    def set_tracking(self, name, value):
        self.trackings[name] = value

    def get_tracking(self, name):
        return self.trackings[name]

    def has_tracking(self, name):
        return name in self.trackings

    def as_tensor_dict(self, fields=None, trackings=None):
        out = {f: self.data[f] for f in (fields or self.data)}
        for t in (trackings if trackings is not None else self.trackings):
            out[t] = self.trackings[t]
        return out

    @classmethod
    def from_tensor_dict(cls, d, fields=None, trackings=None):
        d = dict(d)
        bl = cls(d.pop("boxes"))
        for t in trackings or []:
            bl.set_tracking(t, d.pop(t))
        for f in fields or list(d):
            bl.add_field(f, d[f])
        return bl


class SparseBoxList:
    """indices [M, 2] (image, slot) into a dense [N, P] layout + a BoxList of
    the M valid rows (box_list.py:181-264)."""

    def __init__(self, indices, data, dense_shape):
        assert isinstance(data, BoxList)
        self.indices = indices
        self.data = data
        self.dense_shape = tuple(int(x) for x in dense_shape)
        self.trackings = {}

    def set_tracking(self, name, value):
        self.trackings[name] = value

    def get_tracking(self, name):
        return self.trackings[name]

    def to_dense(self):
        N, P = self.dense_shape
        flat = self.indices[:, 0] * P + self.indices[:, 1]
        out = {}
        for f, v in self.data.data.items():
            if f == "is_valid":
                continue
            dense = torch.zeros((N * P,) + tuple(v.shape[1:]), dtype=v.dtype, device=v.device)
            dense[flat] = v
            out[f] = dense.reshape((N, P) + tuple(v.shape[1:]))
        valid = torch.zeros(N * P, dtype=torch.bool, device=self.indices.device)
        valid[flat] = True
        out["is_valid"] = valid.reshape(N, P)
        dense = BoxList.from_tensor_dict(out)
        for t, v in self.trackings.items():
            dense.set_tracking(t, v)
        return dense

    @classmethod
    def from_dense(cls, boxlist):
        """tf.where(is_valid) + gather_nd: synchronises to learn M."""
        valid = boxlist.get_field("is_valid")
        idx = torch.nonzero(valid)
        data = {f: v[idx[:, 0], idx[:, 1]] for f, v in boxlist.data.items() if f != "is_valid"}
        sp = cls(idx, BoxList.from_tensor_dict(data), valid.shape)
        for t, v in boxlist.trackings.items():
            sp.set_tracking(t, v)
        return sp


class ImageList:
    """Padded batch of NHWC images + true per-image (h, w) (image_list.py:7-101)."""

    def __init__(self, tensor, image_shapes):
        self.tensor = tensor
        self.image_shapes = image_shapes

    @property
    def num_images(self):
        return self.tensor.shape[0]

    @classmethod
    def from_tensors(cls, tensors, image_shapes, size_divisibility=0, pad_value=0.0):
        if pad_value != 0:
            N, H, W = tensors.shape[:3]
            ys = torch.arange(H, device=tensors.device)[None, :, None]
            xs = torch.arange(W, device=tensors.device)[None, None, :]
            hw = image_shapes.to(tensors.device)
            inside = (ys < hw[:, 0, None, None]) & (xs < hw[:, 1, None, None])
            tensors = torch.where(inside[..., None], tensors, torch.full_like(tensors, pad_value))
        if size_divisibility > 0:
            H, W = tensors.shape[1:3]
            s = size_divisibility
            ph, pw = (-H) % s, (-W) % s
            if ph or pw:
                tensors = torch.nn.functional.pad(tensors, (0, 0, 0, pw, 0, ph), value=pad_value)
        return cls(tensors, image_shapes)
