class Box:
  def __init__(self, *a, **k):
    self.args, self.kwargs = a, k
