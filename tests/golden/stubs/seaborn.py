"""Stand-in for seaborn (imported, unused on the scored path)."""
