"""Framework utilities: flat parameter storage, checkpoint/resume, metrics, tracing, config."""
