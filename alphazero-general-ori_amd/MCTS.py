"""Drop-in for the reference's `from MCTS import MCTS` (MCTS.py): device-resident search."""
from splendor.search import MCTS  # noqa: F401
