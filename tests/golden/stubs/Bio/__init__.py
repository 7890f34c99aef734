"""Stand-in for Biopython used ONLY when running the reference scripts for golden vectors."""
