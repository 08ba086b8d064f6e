"""Graph transforms used by the conv modules (``python/dgl/transform.py``)."""
import numpy as np


def laplacian_lambda_max(g):
    """Largest eigenvalue of I - D^-1/2 A D^-1/2 (in-degree norm, clipped at 1) per
    graph, as a list (``transform.py:396-434``; an unbatched graph is a batch of
    one).  Host scipy ``eigs`` as the reference -- setup work, not on the
    message-passing path."""
    from scipy import sparse
    from scipy.sparse import linalg
    n = g.number_of_nodes()
    adj = g.adjacency_matrix_scipy().astype(float)
    deg = np.asarray(g.in_degrees().numpy(), dtype=float).clip(1)
    norm = sparse.diags(deg ** -0.5, dtype=float)
    lap = sparse.eye(n) - norm * adj * norm
    return [float(linalg.eigs(lap, 1, which="LM", return_eigenvectors=False)[0].real)]
