class BatchTracer:  # sentinel isinstance target
  pass
