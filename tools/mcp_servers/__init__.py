import tools  # noqa: F401  (puts the repo root on sys.path)
