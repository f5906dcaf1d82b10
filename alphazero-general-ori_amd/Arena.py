"""Drop-in for the reference's `from Arena import Arena` (Arena.py): same constructor and
playGame / playGames over the engine-backed Game API; splendor.arena.BatchedArena plays the
Coach's new-vs-previous gate on device trees."""
from splendor.arena import Arena, BatchedArena  # noqa: F401
