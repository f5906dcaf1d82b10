"""Drop-in for the reference's `from Coach import Coach` (Coach.py): batched device self-play."""
from splendor.coach import Coach  # noqa: F401
