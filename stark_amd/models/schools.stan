// Eight schools, non-centred parameterisation (the model of stark's example and test,
// example/schools.stan in randommm/stark).  Flat priors on mu and tau.
data {
  int<lower=0> J;           // number of schools
  real y[J];                // estimated treatment effects
  real<lower=0> sigma[J];   // standard errors
}
parameters {
  real mu;
  real<lower=0> tau;
  real eta[J];
}
transformed parameters {
  real theta[J];
  for (j in 1:J)
    theta[j] = mu + tau * eta[j];
}
model {
  eta ~ normal(0, 1);
  y ~ normal(theta, sigma);
}
