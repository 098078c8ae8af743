// Bayesian logistic regression with normal(0, s) priors on the intercept and the coefficients.
data {
  int<lower=0> N;
  int<lower=0> K;
  matrix[N, K] x;
  int<lower=0, upper=1> y[N];
}
parameters {
  real alpha;
  vector[K] beta;
}
model {
  alpha ~ normal(0, 2.5);
  beta ~ normal(0, 1);
  y ~ bernoulli_logit(alpha + x * beta);
}
