"""Restatement of vector_quantize_pytorch 1.17.8 ResidualFSQ (inference path used by the
reference decoder: get_output_from_indices)."""
import torch


class FSQ(torch.nn.Module):
    def __init__(self, levels):
        super().__init__()
        lv = torch.tensor(levels, dtype=torch.int32)
        self.register_buffer("_levels", lv, persistent=False)
        basis = torch.cumprod(torch.tensor([1] + list(levels[:-1])), dim=0, dtype=torch.int32)
        self.register_buffer("_basis", basis, persistent=False)
        self.codebook_size = int(torch.prod(lv))
        self.register_buffer("implicit_codebook", self._indices_to_codes(torch.arange(self.codebook_size)),
                             persistent=False)

    def _indices_to_codes(self, indices):
        level_indices = (indices[..., None] // self._basis) % self._levels
        half_width = self._levels // 2
        return (level_indices - half_width) / half_width


class ResidualFSQ(torch.nn.Module):
    def __init__(self, *, levels, num_quantizers, dim=None, **kwargs):
        super().__init__()
        codebook_dim = len(levels)
        dim = dim if dim is not None else codebook_dim
        self.project_in = torch.nn.Linear(dim, codebook_dim) if dim != codebook_dim else torch.nn.Identity()
        self.project_out = torch.nn.Linear(codebook_dim, dim) if dim != codebook_dim else torch.nn.Identity()
        self.layers = torch.nn.ModuleList([FSQ(levels) for _ in range(num_quantizers)])
        lt = torch.tensor(levels, dtype=torch.float32)
        self.register_buffer("scales", torch.stack([(lt - 1) ** -q for q in range(num_quantizers)]),
                             persistent=False)

    @property
    def codebooks(self):
        return torch.stack([layer.implicit_codebook for layer in self.layers])

    def get_codes_from_indices(self, indices):
        # indices: [b, n, q] -> codes [q, b, n, d]
        q = indices.shape[-1]
        cb = self.codebooks[:q]
        codes = torch.stack([cb[i][indices[..., i]] for i in range(q)])
        return codes * self.scales[:q].view(q, 1, 1, -1)

    def get_output_from_indices(self, indices):
        codes = self.get_codes_from_indices(indices)
        return self.project_out(codes.sum(0))
